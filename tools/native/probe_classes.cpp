// Measurement tool derived from tests/native/diamond_model.cpp: of the probes left
// after commuting diamonds, how many two candidate same-parent rules would remove
// (A: a Receive equal to Drop of its message; B: an UpdateTerm equal to an earlier
// slot one).  // Host model of commuting-diamond probe elimination.
//
// A BFS on the packed encoding (raft_packed.h, the kernels' own lane code),
// recording for every stored state t its first discoverer: parent s and lane
// a, t = a(s).  When t is expanded, a successor b(t) need not be probed when
//   (1) b precedes a in a fixed, state-independent order of action instances
//       (family, then the lane index for server actions, the message for bag
//       actions);
//   (2) a and b are independent: they read/write different server words
//       (a lane touches at most one: Restart..AppendEntries their server i,
//       Receive the message's mdest, Duplicate/Drop none) and touch disjoint
//       messages (the message acted on, the message added);
//   (3) b(s) satisfies the CONSTRAINT (only |DOMAIN messages| can differ from
//       b(t): by a's net change of the bag's domain).
// Then b is enabled at s with the same effect, a is enabled at b(s), and
// a(b(s)) = b(a(s)) = b(t): the state is generated from b(s), a state of the
// same or an earlier level, in the same or an earlier pass.  Successors whose
// probe is skipped still count as generated (TLC counts them).  Mode "check"
// runs the BFS twice, without and with skipping, and requires identical
// per-level counts; mode "count" reports the skippable fraction of probes.
// Build: g++ -O2 -std=c++17 -I raft.tla_amd/csrc diamond_model.cpp
// Run:   ./a.out S V MaxTerm MaxLogLen MaxMsgs MaxDup max_levels
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "raft_packed.h"

using namespace rmc;

namespace {

struct Foot {  // what the kernels would store per state: the discovering lane's messages
    u32 m_act;   // message acted on (Receive / Duplicate / Drop), 0 otherwise
    u32 m_add;   // message added, 0 when none
    uint8_t consumed, has_add, has_act;
};

template <int S, int K>
struct Model {
    Params P{};
    int nl = Lanes<S, K>::N;
    std::vector<u64> W;      // S words per state
    std::vector<u32> M;      // K slots per state
    std::vector<uint8_t> act;
    std::vector<Foot> foot;
    std::vector<u64> hfoot;  // the kernels' footprint word (make_foot)
    std::vector<u64> table;
    u64 mask = 0;

    int family(int lane) const {
        int f = 0;
        while (f < 9 && lane >= P.off[f + 1]) ++f;
        return f;
    }
    u64 last_slot = 0;
    bool insert(u64 key) {
        key = key ? key : 1;
        for (u64 s = key & mask;; s = (s + 1) & mask) {
            if (table[s] == key) { last_slot = s; return false; }
            if (!table[s]) { table[s] = key; last_slot = s; return true; }
        }
    }
    // the server word a lane reads/writes (-1: none) and the message it acts on
    int lane_server(int lane, u32 msg) const {
        const int f = family(lane);
        const int t = lane - P.off[f];
        switch (f) {
            case 0: case 1: case 3: case 5: return t;
            case 2: case 6: return t / S;
            case 4: return t / VMAX;
            case 7: return (int)m_dst(msg);
            default: return -1;
        }
    }
    int rank[10] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9};  // family order of the diamond rule (argv 9)
    u64 order_key(int lane, u32 msg) const {
        const int f = family(lane);
        return ((u64)rank[f] << 40) | (f < 7 ? (u64)lane : (u64)(msg & MSG_MASK));
    }
    static int cnt_of(const u32 (&m)[K], u32 msg) {
        for (int q = 0; q < K; ++q)
            if (m[q] && (m[q] & MSG_MASK) == msg) return (int)m_cnt(m[q]);
        return 0;
    }
    // |DOMAIN messages| of the successor of delta d on (w, m)
    static int dom_after(const u32 (&m)[K], const Delta& d) {
        int n = 0;
        for (int q = 0; q < K; ++q) n += m[q] ? 1 : 0;
        if (d.rm >= 0 && m_cnt(selm<K>(m, d.rm)) <= 1) n -= 1;
        if (d.has_add && !cnt_of(m, d.add)) n += 1;
        return n;
    }
    bool skippable(u64 t, const u32 (&m)[K], int lane_b, const Delta& db) const {
        const int a = act[t];
        if (a == 255) return false;
        const Foot& fa = foot[t];
        const int fb = family(lane_b);
        const u32 mb = fb >= 7 ? (selm<K>(m, lane_b - P.off[fb]) & MSG_MASK) : 0u;
        // (1) order
        if (!(order_key(lane_b, mb) < order_key(a, fa.m_act))) return false;
        // (2) independence: server words
        const int sa = lane_server(a, fa.m_act), sb = lane_server(lane_b, mb);
        if (sa >= 0 && sb >= 0 && sa == sb) return false;
        // (2) independence: messages
        u32 ka[2], kb[2];
        int na = 0, nb = 0;
        if (fa.has_act) ka[na++] = fa.m_act;
        if (fa.has_add) ka[na++] = fa.m_add;
        if (fb >= 7) kb[nb++] = mb;
        if (db.has_add) kb[nb++] = db.add;
        for (int x = 0; x < na; ++x)
            for (int y = 0; y < nb; ++y)
                if (ka[x] == kb[y]) return false;
        // (3) b(s) in the model: |DOMAIN| differs from b(t)'s by a's net domain change
        int delta_a = 0;
        if (fa.has_add && cnt_of(m, fa.m_add) == 1) delta_a += 1;   // a created the key
        if (fa.consumed && cnt_of(m, fa.m_act) == 0) delta_a -= 1;  // a removed its last copy
        if (dom_after(m, db) - delta_a > P.max_msgs) return false;
        return true;
    }

    struct Out {
        std::vector<u64> level_new;
        u64 generated = 0, probes = 0, skipped = 0, mismatch = 0;
        u64 hits = 0, ruleA = 0, ruleA_hit = 0, ruleB = 0, ruleB_hit = 0, ruleC = 0, ruleC_hit = 0, ruleD = 0, ruleD_hit = 0;
        u64 hit_rel[4] = {0, 0, 0, 0};  // found state's level - parent level + 2 (0: <= -2)
        u64 hit_fam[10] = {0}, probe_fam[10] = {0};
    };
    std::vector<u64> slot_idx;  // table slot -> state index
    std::vector<int> lvl_of;    // state index -> level

    Out bfs(int max_levels, bool skip, u64 cap) {
        Out o;
        W.clear(); M.clear(); act.clear(); foot.clear(); hfoot.clear();
        u64 slots = 1;
        while (slots < 2 * cap) slots <<= 1;
        table.assign(slots, 0);
        slot_idx.assign(slots, 0);
        lvl_of.clear();
        mask = slots - 1;
        u64 w0[S];
        u32 m0[K];
        for (int i = 0; i < S; ++i) w0[i] = 1ull | ((u64)NILV << VF_SH);
        for (int q = 0; q < K; ++q) m0[q] = 0;
        insert(state_fp<S, K>(w0, m0).k);
        slot_idx[last_slot] = 0;
        lvl_of.push_back(1);
        W.insert(W.end(), w0, w0 + S);
        M.insert(M.end(), m0, m0 + K);
        act.push_back(255);
        foot.push_back(Foot{});
        hfoot.push_back(0);
        o.generated = 1;
        o.level_new.push_back(1);
        u64 lo = 0, hi = 1;
        for (int lv = 1; (max_levels == 0 || lv < max_levels) && lo < hi; ++lv) {
            for (u64 t = lo; t < hi; ++t) {
                u64 w[S];
                u32 m[K];
                for (int i = 0; i < S; ++i) w[i] = W[t * S + i];
                for (int q = 0; q < K; ++q) m[q] = M[t * K + q];
                const Fp h0 = state_fp<S, K>(w, m);
                ParentMix<S, K> pm;
                parent_mix<S, K>(w, m, pm);
                for (int lane = 0; lane < nl; ++lane) {
                    Delta d;
                    lane_delta<S, K>(w, m, lane, P, d);
                    {  // the descriptor path of the sorted kernels gives the same delta
                        Delta dd;
                        lane_delta_desc<S, K>(w, m, P.ldesc[lane], P, dd);
                        if (dd.en != d.en || dd.srv != d.srv || dd.rm != d.rm || dd.has_add != d.has_add ||
                            (d.en && (dd.w_new != d.w_new || dd.add != d.add)))
                            ++o.mismatch;
                    }
                    if (!d.en) continue;
                    ++o.generated;
                    Fp h{0, 0};
                    {  // the kernels' precomputed-mix form decides and hashes the same (both sums)
                        Fp hp{0, 0}, hf{0, 0};
                        int np = 0, nf = 0;
                        const int a1 = delta_fp<S, K>(w, m, h0, d, P, &hf, &nf);
                        const int a2 = delta_fp_pre<S, K>(w, m, pm, d, P, &hp, &np);
                        if (a1 != a2 || (a1 && (hf.k != hp.k || hf.s != hp.s || nf != np))) ++o.mismatch;
                    }
                    if (!delta_fp<S, K>(w, m, h0, d, P, &h)) continue;
                    {  // the incremental sums equal the materialised successor's (both sums)
                        u64 wo[S];
                        u32 mo[K];
                        materialise<S, K>(w, m, d, wo, mo);
                        const Fp hm = state_fp<S, K>(wo, mo);
                        if (hm.k != h.k || hm.s != h.s) ++o.mismatch;
                    }
                    if (h.k == h0.k) continue;  // stutter
                    const bool sk = skippable(t, m, lane, d);
                    {  // the kernels' implementation (raft_packed.h) must decide the same
                        Diamond dm;
                        diamond_of<S, K>(m, act[t], hfoot[t], P, dm);
                        int nmb = 0;
                        Fp h2{0, 0};
                        delta_fp<S, K>(w, m, h0, d, P, &h2, &nmb);
                        (void)nmb;
                    }
                    if (sk) {
                        ++o.skipped;
                        if (skip) continue;
                    }
                    ++o.probes;
                    const int fam = family(lane);
                    // rule A: a Receive whose successor is Drop(k)'s (no word change, no add, slot k removed)
                    bool rA = false, rB = false;
                    if (fam == 7) {
                        const int k = lane - P.off[7];
                        const bool noword = d.srv < 0 || d.w_new == selw<S>(w, d.srv);
                        rA = d.rm == k && !d.has_add && noword;
                        // rule B: an UpdateTerm (word change only) equal to an earlier slot's UpdateTerm
                        if (d.rm < 0 && !d.has_add && d.srv >= 0)
                            for (int k2 = 0; k2 < k; ++k2) {
                                Delta d2;
                                lane_delta<S, K>(w, m, P.off[7] + k2, P, d2);
                                if (d2.en && d2.rm < 0 && !d2.has_add && d2.srv == d.srv && d2.w_new == d.w_new) rB = true;
                            }
                    }
                    // rule C: Drop(m) undoing the discovering lane's pure add of m (RequestVote,
                    // AppendEntries, DuplicateMessage): the successor is t's parent
                    bool rC = false;
                    if (fam == 9 && act[t] != 255) {
                        const int fa = family(act[t]);
                        const u32 mb = selm<K>(m, lane - P.off[9]) & MSG_MASK;
                        rC = (fa == 2 || fa == 6 || fa == 8) && foot[t].has_add && foot[t].m_add == mb;
                        if (fa == 8) rC = foot[t].has_act && foot[t].m_act == mb;
                    }
                    // rule D: Restart(i) absorbing the discovering lane's change of server i
                    // (BecomeLeader(i), AdvanceCommitIndex(i): fields Restart resets)
                    bool rD = false;
                    if (fam == 0 && act[t] != 255) {
                        const int fa = family(act[t]);
                        rD = (fa == 3 || fa == 5) && (act[t] - P.off[fa]) == (lane - P.off[0]);
                    }
                    const bool fresh = insert(h.k);
                    if (rD) { ++o.ruleD; if (!fresh) ++o.ruleD_hit; }
                    if (rC) { ++o.ruleC; if (!fresh) ++o.ruleC_hit; }
                    ++o.probe_fam[fam];
                    if (!fresh) {
                        ++o.hits;
                        ++o.hit_fam[fam];
                        const int rel = lvl_of[slot_idx[last_slot]] - lv;  // parent at level lv
                        ++o.hit_rel[rel <= -2 ? 0 : rel + 2 > 3 ? 3 : rel + 2];
                    } else {
                        slot_idx[last_slot] = act.size();
                        lvl_of.push_back(lv + 1);
                    }
                    if (rA) { ++o.ruleA; if (!fresh) ++o.ruleA_hit; }
                    if (rB) { ++o.ruleB; if (!fresh) ++o.ruleB_hit; }
                    if (!fresh) continue;
                    u64 wo[S];
                    u32 mo[K];
                    materialise<S, K>(w, m, d, wo, mo);
                    W.insert(W.end(), wo, wo + S);
                    M.insert(M.end(), mo, mo + K);
                    act.push_back((uint8_t)lane);
                    Foot f{};
                    if (fam >= 7) {
                        f.has_act = 1;
                        f.m_act = selm<K>(m, lane - P.off[fam]) & MSG_MASK;
                        f.consumed = d.rm >= 0;
                    }
                    if (d.has_add) { f.has_add = 1; f.m_add = d.add; }
                    foot.push_back(f);
                    hfoot.push_back(make_foot<S, K>(m, lane, d, P));
                }
            }
            lo = hi;
            hi = act.size();
            if (hi > lo) o.level_new.push_back(hi - lo);
            if (act.size() > cap) { fprintf(stderr, "capacity\n"); exit(2); }
        }
        return o;
    }
};

static const char* g_rank = nullptr;
template <int S, int K>
int run(int V, int mt, int ml, int mm, int md, int levels, u64 cap) {
    Model<S, K> X;
    if (g_rank)
        for (int f = 0; f < 10 && g_rank[f]; ++f) X.rank[g_rank[f] - '0'] = f;  // "9012345678": Drop first
    X.P.V = V; X.P.max_term = mt; X.P.max_log = ml; X.P.max_msgs = mm; X.P.max_dup = md; X.P.diamond = 1;
    for (int f = 0; f <= 10; ++f) X.P.off[f] = Lanes<S, K>::off(f);
    fill_lane_desc(X.P, S);
    auto a = X.bfs(levels, true, cap);
    u64 da = 0;
    for (u64 x : a.level_new) da += x;
    printf("hit level - parent level: <=-2 %llu, -1 %llu, 0 %llu, +1 %llu\n", (unsigned long long)a.hit_rel[0],
           (unsigned long long)a.hit_rel[1], (unsigned long long)a.hit_rel[2], (unsigned long long)a.hit_rel[3]);
    for (int f = 0; f < 10; ++f)
        printf("family %d: probes %llu hits %llu\n", f, (unsigned long long)a.probe_fam[f], (unsigned long long)a.hit_fam[f]);
    printf("skipped by diamonds %llu; rule C %llu (hits %llu); rule D %llu (hits %llu)\n",
           (unsigned long long)a.skipped, (unsigned long long)a.ruleC, (unsigned long long)a.ruleC_hit,
           (unsigned long long)a.ruleD, (unsigned long long)a.ruleD_hit);
    printf("{\"distinct\": %llu, \"generated\": %llu, \"probes\": %llu, \"hits\": %llu, \"ruleA\": %llu, "
           "\"ruleA_hit\": %llu, \"ruleB\": %llu, \"ruleB_hit\": %llu}\n",
           (unsigned long long)da, (unsigned long long)a.generated, (unsigned long long)a.probes,
           (unsigned long long)a.hits, (unsigned long long)a.ruleA, (unsigned long long)a.ruleA_hit,
           (unsigned long long)a.ruleB, (unsigned long long)a.ruleB_hit);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 8) {
        fprintf(stderr, "usage: %s S V MaxTerm MaxLogLen MaxMsgs MaxDup max_levels [capacity]\n", argv[0]);
        return 2;
    }
    const int S = atoi(argv[1]), V = atoi(argv[2]), mt = atoi(argv[3]), ml = atoi(argv[4]), mm = atoi(argv[5]),
              md = atoi(argv[6]), lv = atoi(argv[7]);
    const u64 cap = argc > 8 ? strtoull(argv[8], nullptr, 10) : (1ull << 26);
    if (argc > 9) g_rank = argv[9];
    const bool k8 = mm > 4;
    if (S == 2) return k8 ? run<2, 8>(V, mt, ml, mm, md, lv, cap) : run<2, 4>(V, mt, ml, mm, md, lv, cap);
    if (S == 3) return k8 ? run<3, 8>(V, mt, ml, mm, md, lv, cap) : run<3, 4>(V, mt, ml, mm, md, lv, cap);
    if (S == 4) return k8 ? run<4, 8>(V, mt, ml, mm, md, lv, cap) : run<4, 4>(V, mt, ml, mm, md, lv, cap);
    return k8 ? run<5, 8>(V, mt, ml, mm, md, lv, cap) : run<5, 4>(V, mt, ml, mm, md, lv, cap);
}
