// Host check of the incremental SYMMETRY keys (raft_packed.h canon_delta_inc)
// against the whole-successor form (canon_delta<S, K, true>): random walks
// from Init through the packed successor code; at every visited state every
// in-model lane must give the same tie flag and, untied, the same key.
// Build: g++ -O2 -std=c++17 -I raft.tla_amd/csrc sym_inc_check.cpp
// Run:   ./a.out <walks> <depth> <seed>   (prints "ok <lanes checked> ..." or the first mismatch)
#include <cstdio>
#include <cstdlib>

#include "raft_packed.h"

using namespace rmc;

static u64 rng(u64& x) {
    x += 0x9E3779B97F4A7C15ull;
    return mix64(x);
}

template <int S, int K>
static int run(u64 walks, int depth, u64 seed, u64* lanes_checked, u64* same_frame) {
    Params P{};
    P.V = 2; P.max_term = 6; P.max_log = 3; P.max_msgs = K; P.max_dup = 3;
    for (int f = 0; f <= 10; ++f) P.off[f] = Lanes<S, K>::off(f);
    const int nl = Lanes<S, K>::N;
    u64 x = seed;
    for (u64 wk = 0; wk < walks; ++wk) {
        u64 w[S];
        u32 m[K];
        for (int i = 0; i < S; ++i) w[i] = 1ull | ((u64)NILV << VF_SH);  // Init: term 1, Follower, Nil
        for (int q = 0; q < K; ++q) m[q] = 0;
        for (int dd = 0; dd < depth; ++dd) {
            u64 base[S];
            for (int i = 0; i < S; ++i) base[i] = sig_base<S>(w[i], (u32)i);
            SymParent<S, K> sp;
            sym_parent<S, K>(w, m, base, sp);
            int cand[64], nc = 0;
            for (int lane = 0; lane < nl; ++lane) {
                Delta d;
                lane_delta<S, K>(w, m, lane, P, d);
                if (!d.en || !delta_in_model<S, K>(m, d, P)) continue;
                cand[nc++] = lane;
                int t0 = 0, t1 = 0;
                const u64 a = canon_delta<S, K, true>(w, m, base, d, nullptr, 0, &t0);
                const u64 b = canon_delta_inc<S, K>(w, m, base, sp, d, nullptr, 0, &t1);
                ++*lanes_checked;
                if (!t0) {  // does the successor sort by the parent's permutation (the cheap path)?
                    u64 wo[S], bo[S];
                    u32 mo[K], lo, tc;
                    materialise<S, K>(w, m, d, wo, mo);
                    for (int i = 0; i < S; ++i) bo[i] = sig_base<S>(wo[i], (u32)i);
                    Sig<S> sg;
                    signatures<S, K>(bo, mo, sg);
                    sig_rank<S>(sg, &lo, &tc);
                    *same_frame += lo == sp.lo ? 1u : 0u;
                }
                if (t0 != t1 || (!t0 && a != b)) {
                    printf("MISMATCH S=%d K=%d walk %llu depth %d lane %d: tie %d/%d key %016llx/%016llx\n", S, K,
                           (unsigned long long)wk, dd, lane, t0, t1, (unsigned long long)a, (unsigned long long)b);
                    return 1;
                }
            }
            if (!nc) break;
            const int lane = cand[rng(x) % (u64)nc];
            Delta d;
            lane_delta<S, K>(w, m, lane, P, d);
            u64 wo[S];
            u32 mo[K];
            materialise<S, K>(w, m, d, wo, mo);
            for (int i = 0; i < S; ++i) w[i] = wo[i];
            for (int q = 0; q < K; ++q) m[q] = mo[q];
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    const u64 walks = argc > 1 ? strtoull(argv[1], nullptr, 10) : 2000;
    const int depth = argc > 2 ? atoi(argv[2]) : 40;
    const u64 seed = argc > 3 ? strtoull(argv[3], nullptr, 10) : 1;
    u64 n = 0, sf = 0;
    int rc = run<2, 4>(walks, depth, seed, &n, &sf) || run<3, 4>(walks, depth, seed + 1, &n, &sf) ||
             run<3, 8>(walks, depth, seed + 2, &n, &sf) || run<4, 4>(walks, depth, seed + 3, &n, &sf) ||
             run<4, 8>(walks, depth, seed + 4, &n, &sf) || run<5, 4>(walks, depth, seed + 5, &n, &sf) ||
             run<5, 8>(walks, depth, seed + 6, &n, &sf);
    if (rc) return 1;
    printf("ok %llu lanes checked, %llu (%.1f %%) in the parent's frame\n", (unsigned long long)n,
           (unsigned long long)sf, n ? 100.0 * (double)sf / (double)n : 0.0);
    return 0;
}
