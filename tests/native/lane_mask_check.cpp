// Host check of the expansion kernel's lane walk (raft_packed.h lane_superset):
// the mask must contain every lane that lane_delta enables, on every state of
// random walks from Init, for every shape (the sorted kernels run all of them);
// a missing lane would silently drop successors.  Also checks that
// state_class / state_class_fine stay inside their bin ranges.
// Build: g++ -O2 -std=c++17 -I raft.tla_amd/csrc lane_mask_check.cpp
// Run:   ./a.out <walks> <depth> <seed>   (prints "ok ..." or the first failure)
#include <cstdio>
#include <cstdlib>

#include "raft_packed.h"

using namespace rmc;

static u64 rng(u64& x) {
    x += 0x9E3779B97F4A7C15ull;
    return mix64(x);
}

template <int S, int K>
static int run(u64 walks, int depth, u64 seed, int V, u64* checked, u64* lanes_on) {
    Params P{};
    P.V = V; P.max_term = 6; P.max_log = 3; P.max_msgs = K; P.max_dup = 3;
    for (int f = 0; f <= 10; ++f) P.off[f] = Lanes<S, K>::off(f);
    const int nl = Lanes<S, K>::N;
    u64 x = seed;
    for (u64 wk = 0; wk < walks; ++wk) {
        u64 w[S];
        u32 m[K];
        for (int i = 0; i < S; ++i) w[i] = 1ull | ((u64)NILV << VF_SH);
        for (int q = 0; q < K; ++q) m[q] = 0;
        for (int dd = 0; dd < depth; ++dd) {
            const LaneMask mk = lane_superset<S, K>(w, m, V);
            if (state_class<S>(w) >= 64) { printf("state_class out of range\n"); return 1; }
            if (state_class_fine<S, K>(w, m) > 255) { printf("state_class_fine out of range\n"); return 1; }
            int cand[128], nc = 0;
            for (int lane = 0; lane < nl; ++lane) {
                Delta d;
                lane_delta<S, K>(w, m, lane, P, d);
                ++*checked;
                if (!d.en) continue;
                ++*lanes_on;
                if (!mk.has(lane)) {
                    printf("MISSING S=%d K=%d V=%d walk %llu depth %d: lane %d enabled, not in %016llx:%016llx\n", S,
                           K, V, (unsigned long long)wk, dd, lane, (unsigned long long)mk.hi, (unsigned long long)mk.lo);
                    return 1;
                }
                if (delta_in_model<S, K>(m, d, P)) cand[nc++] = lane;
            }
            if (!nc) break;
            Delta d;
            lane_delta<S, K>(w, m, cand[rng(x) % (u64)nc], P, d);
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
    const int depth = argc > 2 ? atoi(argv[2]) : 60;
    const u64 seed = argc > 3 ? strtoull(argv[3], nullptr, 10) : 1;
    u64 n = 0, on = 0;
    for (int V = 1; V <= 2; ++V)
        if (run<2, 4>(walks, depth, seed, V, &n, &on) || run<2, 8>(walks, depth, seed + 1, V, &n, &on) ||
            run<3, 4>(walks, depth, seed + 2, V, &n, &on) || run<3, 8>(walks, depth, seed + 3, V, &n, &on) ||
            run<4, 4>(walks, depth, seed + 4, V, &n, &on) || run<4, 8>(walks, depth, seed + 5, V, &n, &on) ||
            run<5, 4>(walks, depth, seed + 6, V, &n, &on) || run<5, 8>(walks, depth, seed + 7, V, &n, &on))
            return 1;
    printf("ok %llu lanes checked, %llu enabled, all inside lane_superset\n", (unsigned long long)n,
           (unsigned long long)on);
    return 0;
}
