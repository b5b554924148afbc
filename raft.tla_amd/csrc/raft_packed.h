// raft_packed.h — bit-packed raft.tla state and the per-lane successor logic.
//
// One state = S 64-bit server words + K 32-bit bag slots (DESIGN.md "Packed
// state").  Every action of Next (raft.tla:421-430) changes at most ONE server
// word plus at most one bag add and one bag remove, so a lane computes a
// successor as a *delta* against its parent (server index + new word, slot to
// decrement, message to add) and its fingerprint incrementally from the
// parent's.  Only successors that turn out to be new are materialised.
//
// This header is compiled for the host (codec, tests) and for gfx950 (the
// expansion kernels); nothing in it allocates or loops unboundedly.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define RMC_HD __host__ __device__ __forceinline__
#else
#define RMC_HD inline
#endif

namespace rmc {
typedef uint64_t u64;
typedef uint32_t u32;

// ---- server word (raft.tla:37-67, one per server) ---------------------------
//  bits  0-3  currentTerm          bits 11-12 Len(log)
//  bits  4-5  state (F/C/L)        bits 13-27 log[1..3], 5 bits each: term(4) | value(1)<<4
//  bits  6-8  votedFor (7 = Nil)   bits 28..  votesResponded (S), votesGranted (S),
//  bits  9-10 commitIndex                     nextIndex-1 (2 bits x S), matchIndex (2 bits x S)
constexpr int CT_SH = 0, ST_SH = 4, VF_SH = 6, CI_SH = 9, LEN_SH = 11, LOG_SH = 13;
constexpr int ENT_W = 5, LOG_CAP = 3;
constexpr int VR_SH = LOG_SH + LOG_CAP * ENT_W;  // 28
constexpr u32 NILV = 7;
enum : u32 { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
enum : u32 { RVQ = 0, RVP = 1, AEQ = 2, AEP = 3 };  // raft.tla:23-24
// Fields kept by Restart (raft.tla:136-143): currentTerm, votedFor, log.
constexpr u64 RESTART_KEEP = 0xFull | (0x7ull << VF_SH) | (0x1FFFFull << LEN_SH);

template <int S>
struct SL {
    static constexpr int VR = VR_SH, VG = VR_SH + S, NI = VR_SH + 2 * S, MI = VR_SH + 4 * S;
    static constexpr int END = VR_SH + 6 * S;
    static_assert(END <= 59, "server word overflow");
    static constexpr u32 SMASK = (1u << S) - 1;
};

RMC_HD u32 bits(u64 w, int sh, int n) { return (u32)((w >> sh) & ((1ull << n) - 1)); }
RMC_HD u64 setbits(u64 w, int sh, int n, u64 v) {
    const u64 m = ((1ull << n) - 1) << sh;
    return (w & ~m) | ((v << sh) & m);
}
RMC_HD u32 w_ct(u64 w) { return bits(w, CT_SH, 4); }
RMC_HD u32 w_st(u64 w) { return bits(w, ST_SH, 2); }
RMC_HD u32 w_vf(u64 w) { return bits(w, VF_SH, 3); }
RMC_HD u32 w_ci(u64 w) { return bits(w, CI_SH, 2); }
RMC_HD u32 w_len(u64 w) { return bits(w, LEN_SH, 2); }
RMC_HD u32 w_ent(u64 w, u32 k) { return bits(w, LOG_SH + ENT_W * (int)k, ENT_W); }  // k 0-based
RMC_HD u32 ent_term(u32 e) { return e & 15u; }
RMC_HD u32 w_last_term(u64 w) {  // LastTerm raft.tla:84
    const u32 n = w_len(w);
    return n ? ent_term(w_ent(w, n - 1)) : 0u;
}
template <int S> RMC_HD u32 w_vr(u64 w) { return bits(w, SL<S>::VR, S); }
template <int S> RMC_HD u32 w_vg(u64 w) { return bits(w, SL<S>::VG, S); }
template <int S> RMC_HD u32 w_ni(u64 w, u32 j) { return bits(w, SL<S>::NI + 2 * (int)j, 2) + 1u; }
template <int S> RMC_HD u32 w_mi(u64 w, u32 j) { return bits(w, SL<S>::MI + 2 * (int)j, 2); }

// ---- bag slot (raft.tla:31, messages) -----------------------------------------
//  bits 0-1 mtype, 2-4 msource, 5-7 mdest, 8-11 mterm, 12-29 body, 30-31 count (1..3)
//  RVQ body: mlastLogTerm 12-15, mlastLogIndex 16-17
//  RVP body: mvoteGranted 12, mlog 13-29 (= server-word bits 11-27: len + entries)
//  AEQ body: mprevLogIndex+1 12-14 (Smokeraft's -1 included), mprevLogTerm 15-18, Len(mentries) 19,
//            entry 20-24, mcommitIndex 25-26
//  AEP body: msuccess 12, mmatchIndex 13-14
// An empty slot is 0 (a live slot has count >= 1).  Canonical bags are sorted
// descending by slot value, so empty slots come last.
constexpr u32 MSG_MASK = (1u << 30) - 1;
constexpr u32 CNT_ONE = 1u << 30;
RMC_HD u32 m_type(u32 m) { return m & 3u; }
RMC_HD u32 m_src(u32 m) { return (m >> 2) & 7u; }
RMC_HD u32 m_dst(u32 m) { return (m >> 5) & 7u; }
RMC_HD u32 m_term(u32 m) { return (m >> 8) & 15u; }
RMC_HD u32 m_cnt(u32 slot) { return slot >> 30; }
RMC_HD u32 m_hdr(u32 type, u32 src, u32 dst, u32 term) {
    return type | (src << 2) | (dst << 5) | (term << 8);
}

// ---- fingerprint ----------------------------------------------------------------
// fp(s) = sum_i mix(w_i ^ tag_i) + sum_{live slots} mix(slot ^ tag_M)  (mod 2^64)
// A sum of per-component mixes is canonical for the bag (order-free) and can be
// updated in O(changed components) per successor.
RMC_HD u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
// Fingerprint salt (rmc_config.seed): XORed into the low 59 bits of every mix
// input, it selects another member of the hash family, so two BFS runs with
// different seeds that report the same counts rule out fingerprint
// collisions in practice.  Device copy set per run (set_fp_salt); 0 = default.
#if defined(__HIPCC__)
static __constant__ u64 c_fp_salt;  // visible to both passes (HIP_SYMBOL needs the host shadow)
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define RMC_FP_SALT c_fp_salt
#else
#define RMC_FP_SALT 0ull
#endif
// Set epoch (round 6): the tag of the current run's fingerprint-set entries in
// their top 8 bits, epoch << 56, set per run with the salt (set_fp_salt); 0 =
// untagged (the set cleared to 0 before the run: sharded, verification and
// resumed runs).  A slot whose tag is not the run's epoch is empty — the
// entries of earlier runs on the same ctx included — so a run on a ctx whose
// set already holds tagged entries starts without clearing it (rmc_run_bfs:
// every 255th run, and the first, clear it whole).
#if defined(__HIPCC__)
static __constant__ u64 c_set_ep;
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define RMC_SET_EP c_set_ep
#else
#define RMC_SET_EP 0ull
#endif
RMC_HD u64 hS(u64 w, u32 i) { return mix64(w ^ ((u64)(i + 1) << 59) ^ RMC_FP_SALT); }
RMC_HD u64 hM(u32 slot) { return slot ? mix64((u64)slot ^ (0x1Full << 59) ^ RMC_FP_SALT) : 0ull; }

// A state's fingerprint is two order-free sums over its components: k = sum of
// the mixes a (the 64-bit key stored in the fingerprint set, as TLC's FP64) and
// s = sum of smix(a) mod 2^32, a second, nonlinear function of each mix (the
// high half of a 32 x 32-bit product of its two halves: one v_mul_hi_u32).  The
// set's slot is taken from k and the stored value is k ^ (s within the slot
// mask) (fp_value): two distinct states collide only if their k AND those bits
// of s agree, 64 + min(32, log2 slots) bits instead of 64 — at 4.13 G states
// the 64-bit birthday bound alone expects 0.46 collisions (DESIGN.md
// "Fingerprints").
RMC_HD u32 smix(u64 a) {
    return (u32)(((u64)((u32)a ^ 0x9E3779B9u) * (u64)((u32)(a >> 32) ^ 0x7F4A7C15u)) >> 32);
}
struct Fp {
    u64 k;
    u32 s;
};
RMC_HD Fp fp_of(u64 a) { return Fp{a, smix(a)}; }
RMC_HD void fp_add(Fp& h, u64 a) { h.k += a; h.s += smix(a); }
RMC_HD void fp_sub(Fp& h, u64 a) { h.k -= a; h.s -= smix(a); }
// A fingerprint's place in a table of mask + 1 slots: the value stored /
// compared, v = k ^ (s & mask) (never 0, the empty slot; a tagged set replaces
// its top 8 bits by the run's epoch: 56 + min(32, log2 slots) bits), and the first slot
// of its probe sequence, k & mask.  The one fingerprint whose value would be 0
// flips bit 0 of s (fp_norm, in every caller alike), so the slot is always
// (v ^ s) & mask and callers may keep (v, s) only (fp_slot).
RMC_HD u32 fp_norm(u64 k, u32 s32, u64 mask) { return (k ^ ((u64)s32 & mask)) == 0 ? (s32 ^ 1u) : s32; }
RMC_HD u64 fp_v(u64 k, u32 s32n, u64 mask) {
    const u64 v = k ^ ((u64)s32n & mask);
    // a tagged set keeps the low 56 bits (mask < 2^56) under the run's epoch
    return RMC_SET_EP ? (v & ((1ull << 56) - 1)) | RMC_SET_EP : v;
}
// An empty slot: 0, or (tagged set) an entry of another run's epoch.
RMC_HD bool fp_empty(u64 cur) { return RMC_SET_EP ? ((cur ^ RMC_SET_EP) >> 56) != 0 : cur == 0; }
RMC_HD u64 fp_slot(u64 v, u32 s32n, u64 mask) { return (v ^ (u64)s32n) & mask; }
struct TKey {
    u64 v, s0;
};
RMC_HD TKey tkey(const Fp& h, u64 mask) {
    const u32 s = fp_norm(h.k, h.s, mask);
    return TKey{fp_v(h.k, s, mask), h.k & mask};
}

// Owner rank of a fingerprint in sharded mode: its top 32 bits scaled to
// [0, world).  The fingerprint-set slot uses the low bits, so every shard's
// table stays uniformly loaded.
RMC_HD u32 owner_of(u64 key, u32 world) { return (u32)(((key >> 32) * (u64)world) >> 32); }

// ---- model parameters (runtime part) --------------------------------------------
struct Params {
    int V, max_term, max_log, max_msgs, max_dup, bug_quorum, inv_mask, symmetry;
    int off[11];  // family lane offsets (= Lanes<S,K>::off, for host code)
    int diamond;  // 1: commuting-diamond successors are not probed (RMC_DIAMOND=0 turns it off)
    int unbounded;  // fields no CONSTRAINT bounds (1 term, 2 log, 4 msgs, 8 dup): their bound is the packed
                    // capacity, and a successor beyond it is an error (capacity_exceeded), not filtered
    u64 fp_mask;  // full-state verification mode: fingerprint bits kept (~0 = all; fewer only
                  // to provoke collisions in tests, rmc_set_fp_bits)
    u32 ldesc[128];  // per-lane descriptor (lane_desc; every shape has < 128 lanes): family | index in
                     // family << 4 | acting server << 12 (7: none or per message); filled by fill_lane_desc
};

// Lane table: Restart S, Timeout S, RequestVote S^2,
// BecomeLeader S, ClientRequest S*VMAX (lanes with v >= |Value| are never
// enabled), AdvanceCommitIndex S, AppendEntries S^2, Receive K,
// DuplicateMessage K, DropMessage K.  Compile-time, so an unrolled lane loop
// folds each lane's family dispatch away.
constexpr int VMAX = 2;
template <int S, int K>
struct Lanes {
    static constexpr int size(int f) {
        return f == 0 ? S : f == 1 ? S : f == 2 ? S * S : f == 3 ? S : f == 4 ? S * VMAX
             : f == 5 ? S : f == 6 ? S * S : K;
    }
    static constexpr int off(int f) { return f == 0 ? 0 : off(f - 1) + size(f - 1); }
    static constexpr int N = off(10);
};

// A successor relative to its parent.
struct Delta {
    u64 w_new;    // new word of server `srv`
    int srv;      // -1: no server word changes
    int rm;       // bag slot to decrement, -1: none
    u32 add;      // message (30 bits) to add when has_add
    int has_add;
    int en;       // lane enabled (counts as generated)
};

// Runtime-indexed reads of register arrays as AND/OR masks: a select chain
// gets folded by the compiler into a dynamically indexed load, which forces
// the array out of registers into scratch (cdna_hip_programming.md §5.4 r20).
template <int S>
RMC_HD u64 selw(const u64 (&w)[S], int i) {
    u64 r = 0;
#pragma unroll
    for (int k = 0; k < S; ++k) r |= w[k] & (0ull - (u64)(i == k));
    return r;
}
template <int K>
RMC_HD u32 selm(const u32 (&m)[K], int i) {
    u32 r = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) r |= m[k] & (0u - (u32)(i == k));
    return r;
}

// Receive(m) raft.tla:388-403 for bag slot k (message `msg`).  (A branch-free
// form — every case a predicate, its effect a select — measured neutral on the
// bench model and 6-17 % slower on S = 5 and simulation: profiles/r03/ab/.)
template <int S, int K>
RMC_HD void receive_lane(const u64 (&w)[S], u32 msg, int k, Delta& d) {
    const u32 i = m_dst(msg), j = m_src(msg), mterm = m_term(msg), mt = m_type(msg);
    const u64 wi = selw<S>(w, (int)i);
    const u32 ct = w_ct(wi), st = w_st(wi), len = w_len(wi);
    d.srv = (int)i;
    d.w_new = wi;
    if (mterm > ct) {  // UpdateTerm :373-379 — m stays in the bag
        u64 wn = setbits(wi, CT_SH, 4, mterm);
        wn = setbits(wn, ST_SH, 2, FOLLOWER);
        d.w_new = setbits(wn, VF_SH, 3, NILV);
        d.en = 1;
        return;
    }
    if (mt == RVQ) {  // HandleRequestVoteRequest :244-263 (mterm <= ct here)
        const u32 lt = w_last_term(wi);
        const u32 mlt = (msg >> 12) & 15u, mli = (msg >> 16) & 3u;
        const bool log_ok = mlt > lt || (mlt == lt && mli >= len);
        const u32 vf = w_vf(wi);
        const bool grant = mterm == ct && log_ok && (vf == NILV || vf == j);
        if (grant) d.w_new = setbits(wi, VF_SH, 3, j);
        // Reply :102-103 — response carries mlog = log[i] (len + entries bits)
        d.add = m_hdr(RVP, i, j, ct) | ((grant ? 1u : 0u) << 12) | (bits(wi, LEN_SH, 17) << 13);
        d.has_add = 1;
        d.rm = k;
        d.en = 1;
        return;
    }
    if (mt == RVP) {
        d.rm = k;
        d.en = 1;
        if (mterm < ct) return;  // DropStaleResponse :382-385
        // HandleRequestVoteResponse :267-279
        u64 wn = wi | (1ull << (SL<S>::VR + (int)j));
        if ((msg >> 12) & 1u) wn |= 1ull << (SL<S>::VG + (int)j);
        d.w_new = wn;
        return;
    }
    if (mt == AEQ) {  // HandleAppendEntriesRequest :347-356 (mterm <= ct here)
        const u32 pe = (msg >> 12) & 7u, pterm = (msg >> 15) & 15u;  // pe = mprevLogIndex + 1
        const u32 nent = (msg >> 19) & 1u, ent = (msg >> 20) & 31u, mci = (msg >> 25) & 3u;
        const u32 pidx = pe - 1u;  // only read when pe >= 1 (mprevLogIndex >= 0)
        // mprevLogIndex = -1 (Smokeraft.tla:35) fails both disjuncts of logOk
        const bool log_ok = pe == 1u || (pe > 1u && pidx <= len && pterm == ent_term(w_ent(wi, pidx - 1)));
        if (mterm < ct || (st == FOLLOWER && !log_ok)) {  // Reject :281-293
            d.add = m_hdr(AEP, i, j, ct);  // msuccess FALSE, mmatchIndex 0
            d.has_add = 1;
            d.rm = k;
            d.en = 1;
            return;
        }
        if (st == CANDIDATE) {  // ReturnToFollowerState :295-299 — m stays
            d.w_new = setbits(wi, ST_SH, 2, FOLLOWER);
            d.en = 1;
            return;
        }
        if (st != FOLLOWER) return;  // Leader with an equal-term request: no branch
        const u32 index = pidx + 1;
        const bool term_eq = len >= index && ent_term(w_ent(wi, index - 1)) == ent_term(ent);
        if (nent == 0 || term_eq) {
            // AppendEntriesAlreadyDone :301-317; UNCHANGED logVars after
            // commitIndex' = [.. EXCEPT ![i] = m.mcommitIndex] is a TLC
            // equality test: enabled only when mcommitIndex = commitIndex[i].
            if (mci != w_ci(wi)) return;
            d.add = m_hdr(AEP, i, j, ct) | (1u << 12) | ((pidx + nent) << 13);
            d.has_add = 1;
            d.rm = k;
            d.en = 1;
            return;
        }
        if (len >= index) {  // ConflictAppendEntriesRequest :319-325 — drop LAST entry, m stays
            u64 wn = setbits(wi, LOG_SH + ENT_W * (int)(len - 1), ENT_W, 0);
            d.w_new = setbits(wn, LEN_SH, 2, len - 1);
            d.en = 1;
            return;
        }
        if (len == pidx) {  // NoConflictAppendEntriesRequest :327-331 — m stays
            if (len >= (u32)LOG_CAP) {  // Len = 4 > every allowed bound: out of constraint
                d.w_new = setbits(wi, LEN_SH, 2, 3) | (1ull << 63);  // bit 63 marks overflow
            } else {
                u64 wn = setbits(wi, LOG_SH + ENT_W * (int)len, ENT_W, ent);
                d.w_new = setbits(wn, LEN_SH, 2, len + 1);
            }
            d.en = 1;
        }
        return;
    }
    // AEP
    d.rm = k;
    d.en = 1;
    if (mterm < ct) return;  // DropStaleResponse
    // HandleAppendEntriesResponse :360-370 (no Leader guard)
    if ((msg >> 12) & 1u) {
        const u32 mm = (msg >> 13) & 3u;
        u64 wn = setbits(wi, SL<S>::NI + 2 * (int)j, 2, mm);  // nextIndex = mm + 1 (stored -1)
        d.w_new = setbits(wn, SL<S>::MI + 2 * (int)j, 2, mm);
    } else {
        const u32 nis = bits(wi, SL<S>::NI + 2 * (int)j, 2);  // nextIndex - 1
        d.w_new = setbits(wi, SL<S>::NI + 2 * (int)j, 2, nis ? nis - 1 : 0);  // Max({ni-1, 1})
    }
}

// The delta of action instance (family fam, index t in the family; i, j its
// servers: RequestVote / AppendEntries (i, j) = (t / S, t % S), ClientRequest
// (i, v) = (t / VMAX, t % VMAX), the other server actions i = t) on parent (w, m).
// fam is a runtime value (a kernel argument or a per-lane descriptor), so the
// family dispatch stays a branch tree: as compile-time constants the compiler
// if-converts every family into straight-line selects and the kernel needs 4x
// the registers.
template <int S, int K>
RMC_HD void lane_delta_f(const u64 (&w)[S], const u32 (&m)[K], int fam, int t, int i, int j, const Params& P,
                         Delta& d) {
    d.srv = -1;
    d.rm = -1;
    d.has_add = 0;
    d.add = 0;
    d.en = 0;
    d.w_new = 0;
    // fam is wave-uniform in the sorted kernels (scalar branches).  The enabling
    // conditions inside a family stay branches: written as predicates + selects
    // they were neutral on the bench model and 4-17 % slower on S = 5 and
    // simulation (profiles/r03/ab/lane_code_c1_c2_c3_r03t.jsonl)
    switch (fam) {
    case 0: {  // Restart(i) :136-143
        d.srv = i;
        d.w_new = selw<S>(w, i) & RESTART_KEEP;
        d.en = 1;
        break;
    }
    case 1: {  // Timeout(i) :146-154
        const u64 wi = selw<S>(w, i);
        const u32 st = w_st(wi);
        if (st == FOLLOWER || st == CANDIDATE) {
            const u32 ct1 = w_ct(wi) + 1;
            u64 wn = setbits(wi, ST_SH, 2, CANDIDATE);
            wn = setbits(wn, VF_SH, 3, NILV);
            wn &= ~(((u64)SL<S>::SMASK << SL<S>::VR) | ((u64)SL<S>::SMASK << SL<S>::VG));
            wn = setbits(wn, CT_SH, 4, ct1 & 15u) | ((u64)(ct1 >> 4) << 63);  // bit 63: term overflow
            d.srv = i;
            d.w_new = wn;
            d.en = 1;
        }
        break;
    }
    case 2: {  // RequestVote(i, j) :157-166 (no i /= j guard)
        const u64 wi = selw<S>(w, i);
        if (w_st(wi) == CANDIDATE && !((w_vr<S>(wi) >> j) & 1u)) {
            d.add = m_hdr(RVQ, (u32)i, (u32)j, w_ct(wi)) | (w_last_term(wi) << 12) | (w_len(wi) << 16);
            d.has_add = 1;
            d.en = 1;
        }
        break;
    }
    case 3: {  // BecomeLeader(i) :195-203
        const u64 wi = selw<S>(w, i);
        const u32 vg = w_vg<S>(wi);
        const bool ok = P.bug_quorum ? vg != 0u : (2 * __builtin_popcount(vg) > S);
        if (w_st(wi) == CANDIDATE && ok) {
            u64 wn = setbits(wi, ST_SH, 2, LEADER);
            const u64 lenv = w_len(wi);  // nextIndex = Len + 1, stored minus one
            u64 ni = 0;
#pragma unroll
            for (int q = 0; q < S; ++q) ni |= lenv << (2 * q);
            wn = setbits(wn, SL<S>::NI, 2 * S, ni);
            wn = setbits(wn, SL<S>::MI, 2 * S, 0);
            d.srv = i;
            d.w_new = wn;
            d.en = 1;
        }
        break;
    }
    case 4: {  // ClientRequest(i, v) :206-213 (v = j)
        const u64 wi = selw<S>(w, i);
        if (j < P.V && w_st(wi) == LEADER) {
            const u32 len = w_len(wi);
            if (len >= (u32)LOG_CAP) {
                d.w_new = wi | (1ull << 63);  // Len = 4: out of every allowed constraint
            } else {
                u64 wn = setbits(wi, LOG_SH + ENT_W * (int)len, ENT_W, w_ct(wi) | ((u32)j << 4));
                d.w_new = setbits(wn, LEN_SH, 2, len + 1);
            }
            d.srv = i;
            d.en = 1;
        }
        break;
    }
    case 5: {  // AdvanceCommitIndex(i) :219-236
        const u64 wi = selw<S>(w, i);
        if (w_st(wi) == LEADER) {
            const u32 len = w_len(wi);
            u32 best = 0;
            for (u32 idx = 1; idx <= len; ++idx) {
                u32 agree = 1u << i;
#pragma unroll
                for (int q = 0; q < S; ++q) agree |= (w_mi<S>(wi, q) >= idx ? 1u : 0u) << q;
                if (2 * __builtin_popcount(agree) > S) best = idx;  // Max(agreeIndexes)
            }
            u64 wn = wi;
            if (best > 0 && ent_term(w_ent(wi, best - 1)) == w_ct(wi)) wn = setbits(wi, CI_SH, 2, best);
            d.srv = i;
            d.w_new = wn;
            d.en = 1;
        }
        break;
    }
    case 6: {  // AppendEntries(i, j) :171-192
        const u64 wi = selw<S>(w, i);
        if (i != j && w_st(wi) == LEADER) {
            const u32 len = w_len(wi), ni = w_ni<S>(wi, (u32)j);
            const u32 prev = ni - 1;
            const u32 pterm = (prev > 0 && prev <= len) ? ent_term(w_ent(wi, prev - 1)) : 0u;
            const u32 last = len < ni ? len : ni;  // Min({Len(log[i]), nextIndex[i][j]})
            const u32 nent = ni <= last ? 1u : 0u; // SubSeq(log[i], ni, last): 0 or 1 entry
            const u32 ent = nent ? w_ent(wi, ni - 1) : 0u;
            const u32 ci = w_ci(wi), mci = ci < last ? ci : last;
            d.add = m_hdr(AEQ, (u32)i, (u32)j, w_ct(wi)) | ((prev + 1u) << 12) | (pterm << 15) | (nent << 19) |
                    (ent << 20) | (mci << 25);
            d.has_add = 1;
            d.en = 1;
        }
        break;
    }
    case 7: {  // Receive(m) :388-403
        const u32 sl = selm<K>(m, t);
        if (sl) receive_lane<S, K>(w, sl & MSG_MASK, t, d);
        break;
    }
    case 8: {  // DuplicateMessage(m) :410-412
        const u32 sl = selm<K>(m, t);
        if (sl) {
            d.add = sl & MSG_MASK;
            d.has_add = 1;
            d.en = 1;
        }
        break;
    }
    default: {  // DropMessage(m) :415-417
        const u32 sl = selm<K>(m, t);
        if (sl) {
            d.rm = t;
            d.en = 1;
        }
        break;
    }
    }
}

// Compute the delta of lane `lane` (0 <= lane < Lanes<S,K>::N) on parent (w, m).
// The family dispatch is a chain on the offsets read from the kernel argument
// (equal to Lanes<S,K>::off), each branch calling lane_delta_f with a constant
// family, so only that family's body is inlined there (computing the family
// first and switching on it measured 57 % slower on the >64-lane S = 5 kernel).
template <int S, int K>
RMC_HD void lane_delta(const u64 (&w)[S], const u32 (&m)[K], int lane, const Params& P, Delta& d) {
    const int* o = P.off;
    if (lane < o[1]) {
        lane_delta_f<S, K>(w, m, 0, lane, lane, 0, P, d);
    } else if (lane < o[2]) {
        const int t = lane - o[1];
        lane_delta_f<S, K>(w, m, 1, t, t, 0, P, d);
    } else if (lane < o[3]) {
        const int t = lane - o[2];
        lane_delta_f<S, K>(w, m, 2, t, t / S, t % S, P, d);
    } else if (lane < o[4]) {
        const int t = lane - o[3];
        lane_delta_f<S, K>(w, m, 3, t, t, 0, P, d);
    } else if (lane < o[5]) {
        const int t = lane - o[4];
        lane_delta_f<S, K>(w, m, 4, t, t / VMAX, t % VMAX, P, d);
    } else if (lane < o[6]) {
        const int t = lane - o[5];
        lane_delta_f<S, K>(w, m, 5, t, t, 0, P, d);
    } else if (lane < o[7]) {
        const int t = lane - o[6];
        lane_delta_f<S, K>(w, m, 6, t, t / S, t % S, P, d);
    } else if (lane < o[8]) {
        const int t = lane - o[7];
        lane_delta_f<S, K>(w, m, 7, t, 0, 0, P, d);
    } else if (lane < o[9]) {
        const int t = lane - o[8];
        lane_delta_f<S, K>(w, m, 8, t, 0, 0, P, d);
    } else {
        const int t = lane - o[9];
        lane_delta_f<S, K>(w, m, 9, t, 0, 0, P, d);
    }
}

// The same from a lane descriptor (Params.ldesc: lane_desc).
template <int S, int K>
RMC_HD void lane_delta_desc(const u64 (&w)[S], const u32 (&m)[K], u32 desc, const Params& P, Delta& d) {
    const int fam = (int)(desc & 15u), t = (int)((desc >> 4) & 255u);
    lane_delta_f<S, K>(w, m, fam, t, (int)((desc >> 16) & 15u), (int)((desc >> 20) & 15u), P, d);
}

// Apply a delta: fingerprint and CONSTRAINT (parent assumed in-constraint).
// Returns 1 if the successor is in the model; *h receives its fingerprint.
template <int S, int K>
RMC_HD int delta_fp(const u64 (&w)[S], const u32 (&m)[K], const Fp& h0, const Delta& d, const Params& P,
                    Fp* h, int* nmsg_out = nullptr) {
    Fp hh = h0;
    int nmsg = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) nmsg += m[q] ? 1 : 0;
    if (d.srv >= 0) {
        const u64 wo = selw<S>(w, d.srv);
        if ((d.w_new >> 63) != 0) return 0;  // term 16 or Len 4: beyond every bound
        if ((int)w_ct(d.w_new) > P.max_term || (int)w_len(d.w_new) > P.max_log) return 0;
        if (d.w_new != wo) {
            fp_add(hh, hS(d.w_new, (u32)d.srv));
            fp_sub(hh, hS(wo, (u32)d.srv));
        }
    }
    if (d.rm >= 0) {
        const u32 sl = selm<K>(m, d.rm);
        fp_sub(hh, hM(sl));
        if (m_cnt(sl) > 1) fp_add(hh, hM(sl - CNT_ONE));
        else nmsg -= 1;
    }
    if (d.has_add) {
        int found = -1;
#pragma unroll
        for (int q = 0; q < K; ++q) found = (m[q] && (m[q] & MSG_MASK) == d.add) ? q : found;
        if (found >= 0) {
            const u32 sl = selm<K>(m, found);
            if ((int)m_cnt(sl) + 1 > P.max_dup) return 0;
            fp_add(hh, hM(sl + CNT_ONE));
            fp_sub(hh, hM(sl));
        } else {
            if (1 > P.max_dup) return 0;
            nmsg += 1;
            fp_add(hh, hM(d.add | CNT_ONE));
        }
    }
    if (nmsg > P.max_msgs) return 0;
    *h = hh;
    if (nmsg_out) *nmsg_out = nmsg;
    return 1;
}

// The parent's per-component mixes, computed once per expanded state: a lane
// then mixes only the components it creates (the new server word, the
// decremented / incremented / added bag slot), about half of delta_fp's
// mixes, and the hash is the expansion kernel's main VALU cost (a mix64 is
// 17 VALU instructions, six of them quarter-rate 32-bit multiplies).
template <int S, int K>
struct ParentMix {
    u64 hw[S];
    u64 hm[K];
    Fp h0;
    int nmsg;
};
template <int S, int K>
RMC_HD void parent_mix(const u64 (&w)[S], const u32 (&m)[K], ParentMix<S, K>& pm) {
    pm.h0 = Fp{0, 0};
    pm.nmsg = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) { pm.hw[i] = hS(w[i], (u32)i); fp_add(pm.h0, pm.hw[i]); }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        pm.hm[q] = hM(m[q]);
        if (m[q]) fp_add(pm.h0, pm.hm[q]);
        pm.nmsg += m[q] ? 1 : 0;
    }
}
template <int N>
RMC_HD u64 sel64(const u64 (&a)[N], int i) {
    u64 r = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) r |= a[k] & (0ull - (u64)(i == k));
    return r;
}
// delta_fp with the parent's mixes precomputed: same result, fewer mixes.
template <int S, int K>
RMC_HD int delta_fp_pre(const u64 (&w)[S], const u32 (&m)[K], const ParentMix<S, K>& pm, const Delta& d,
                        const Params& P, Fp* h, int* nmsg_out = nullptr, u64* hw_new = nullptr) {
    // early returns on purpose: a branch-light form (bounds as predicates, only
    // the mixes under branches) measured 306 vs 289-294 ms per MCraftBench BFS —
    // out-of-model lanes then pay for the whole computation
    Fp hh = pm.h0;
    int nmsg = pm.nmsg;
    if (d.srv >= 0) {
        if ((d.w_new >> 63) != 0) return 0;  // term 16 or Len 4: beyond every bound
        if ((int)w_ct(d.w_new) > P.max_term || (int)w_len(d.w_new) > P.max_log) return 0;
        const u64 wo = selw<S>(w, d.srv);
        const u64 ho = sel64<S>(pm.hw, d.srv);
        const u64 hn = d.w_new != wo ? hS(d.w_new, (u32)d.srv) : ho;
        if (hn != ho) {
            fp_add(hh, hn);
            fp_sub(hh, ho);
        }
        if (hw_new) *hw_new = hn;  // the new word's mix (the sharded owner reuses it)
    }
    if (d.rm >= 0) {
        const u32 sl = selm<K>(m, d.rm);
        fp_sub(hh, sel64<K>(pm.hm, d.rm));
        if (m_cnt(sl) > 1) fp_add(hh, hM(sl - CNT_ONE));
        else nmsg -= 1;
    }
    if (d.has_add) {
        int found = -1;
#pragma unroll
        for (int q = 0; q < K; ++q) found = (m[q] && (m[q] & MSG_MASK) == d.add) ? q : found;
        if (found >= 0) {
            const u32 sl = selm<K>(m, found);
            if ((int)m_cnt(sl) + 1 > P.max_dup) return 0;
            fp_add(hh, hM(sl + CNT_ONE));
            fp_sub(hh, sel64<K>(pm.hm, found));
        } else {
            if (1 > P.max_dup) return 0;
            nmsg += 1;
            fp_add(hh, hM(d.add | CNT_ONE));
        }
    }
    if (nmsg > P.max_msgs) return 0;
    *h = hh;
    if (nmsg_out) *nmsg_out = nmsg;
    return 1;
}

// ---- wave homogeneity (the expansion kernels' window sort) ------------------------------
// A wave walks every action lane that ANY of its 64 states enables, so states
// of one kind (same roles, same number of messages) should sit together.
// state_class_fine: a byte that groups states by the servers' roles and the
// number of messages; every new state's class is stored next to it (B.cls,
// one byte) when it is created, and the expansion kernel counting-sorts its
// windows by it, reading 1 B per state instead of the state.  lane_superset:
// the lanes a state can possibly enable (role and slot occupancy only; a
// superset of the enabled lanes); OR-ed over a wave it is the set of lanes the
// wave must walk.  Both are layout hints: the search is the same whatever they
// return, as long as lane_superset is a superset.
// The class of a stored state (the window sort of the expansion kernel): the
// servers' roles, < 64 values (S <= 3: base-3 digits; else leader mask and
// whether some server is a candidate).
template <int S>
RMC_HD u32 state_class(const u64* ws) {
    u32 roles = 0, lead = 0, cand = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const u32 st = w_st(ws[i]);
        roles = roles * 3u + st;
        lead |= (st == LEADER ? 1u : 0u) << i;
        cand |= st == CANDIDATE ? 1u : 0u;
    }
    if constexpr (S <= 3) return roles;
    return lead | (cand << S);
}
// The window-sort class (< 256): the roles and the number of messages, whose
// slots decide the Receive / Duplicate / Drop lanes a state enables.
template <int S, int K>
RMC_HD u32 state_class_fine(const u64 (&w)[S], const u32 (&m)[K]) {
    int nmsg = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) nmsg += m[q] ? 1 : 0;
    const u32 c = state_class<S>(w);
    if constexpr (S <= 3) return c * 9u + (u32)(nmsg < 8 ? nmsg : 8);  // <= 242
    return c | ((u32)(nmsg < 3 ? nmsg : 3) << (S + 1));                 // S + 3 <= 8 bits
}
// A set of lanes (every shape has fewer than 128): bit l of lo (l < 64) or of hi.
struct LaneMask {
    u64 lo, hi;
    RMC_HD bool has(int l) const { return l < 64 ? ((lo >> l) & 1ull) != 0 : ((hi >> (l - 64)) & 1ull) != 0; }
    // OR in `bits` shifted left by sh (sh and the bits' width are compile-time in the callers)
    RMC_HD void put(u64 bits, int sh) {
        if (sh < 64) {
            lo |= bits << sh;
            if (sh > 0) hi |= bits >> (64 - sh);
        } else {
            hi |= bits << (sh - 64);
        }
    }
};
template <int S, int K>
RMC_HD LaneMask lane_superset(const u64 (&w)[S], const u32 (&m)[K], int V) {
    typedef Lanes<S, K> L;
    static_assert(L::N <= 128, "lane mask holds < 128 lanes");
    // constant expressions: off() is recursive, so a plain call is not folded
    constexpr int O1 = L::off(1), O2 = L::off(2), O3 = L::off(3), O4 = L::off(4), O5 = L::off(5), O6 = L::off(6),
                  O7 = L::off(7), O8 = L::off(8), O9 = L::off(9);
    constexpr u64 SM = (1ull << S) - 1;
    LaneMask mk{SM, 0ull};  // Restart(i): always enabled
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const u32 st = w_st(w[i]);
        if (st != LEADER) mk.put(1ull, O1 + i);                                   // Timeout
        if (st == CANDIDATE) { mk.put(SM, O2 + i * S); mk.put(1ull, O3 + i); }    // RequestVote, BecomeLeader
        if (st == LEADER) {  // ClientRequest, AdvanceCommitIndex, AppendEntries
            mk.put((1ull << V) - 1, O4 + i * VMAX);
            mk.put(1ull, O5 + i);
            mk.put(SM, O6 + i * S);
        }
    }
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (m[q]) { mk.put(1ull, O7 + q); mk.put(1ull, O8 + q); mk.put(1ull, O9 + q); }
    return mk;
}

// CONSTRAINT of a delta without its fingerprint (the SYMMETRY kernels hash the
// canonical form instead).
template <int S, int K>
RMC_HD int delta_in_model(const u32 (&m)[K], const Delta& d, const Params& P) {
    int nmsg = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) nmsg += m[q] ? 1 : 0;
    if (d.srv >= 0) {
        if ((d.w_new >> 63) != 0) return 0;
        if ((int)w_ct(d.w_new) > P.max_term || (int)w_len(d.w_new) > P.max_log) return 0;
    }
    if (d.rm >= 0 && m_cnt(selm<K>(m, d.rm)) <= 1) nmsg -= 1;
    if (d.has_add) {
        int found = -1;
#pragma unroll
        for (int q = 0; q < K; ++q) found = (m[q] && (m[q] & MSG_MASK) == d.add) ? q : found;
        if (found >= 0) {
            if ((int)m_cnt(selm<K>(m, found)) + 1 > P.max_dup) return 0;
        } else {
            if (1 > P.max_dup) return 0;
            nmsg += 1;
        }
    }
    return nmsg <= P.max_msgs;
}

// The unbounded fields (Params.unbounded) a delta takes past the packed
// capacity: 0 = none (the successor is in the model or filtered by a real
// CONSTRAINT), else the field bits.
template <int S, int K>
RMC_HD int capacity_exceeded(const u32 (&m)[K], const Delta& d, const Params& P) {
    int bad = 0;
    if (d.srv >= 0) {  // from an in-model parent (term <= 14) bit 63 only marks a 4th log entry
        if ((P.unbounded & 1) && (d.w_new >> 63) == 0 && (int)w_ct(d.w_new) > P.max_term) bad |= 1;
        if ((P.unbounded & 2) && ((d.w_new >> 63) != 0 || (int)w_len(d.w_new) > P.max_log)) bad |= 2;
    }
    int nmsg = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) nmsg += m[q] ? 1 : 0;
    if (d.rm >= 0 && m_cnt(selm<K>(m, d.rm)) <= 1) nmsg -= 1;
    if (d.has_add) {
        u32 cnt = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) cnt |= (m[q] && (m[q] & MSG_MASK) == d.add) ? m_cnt(m[q]) : 0u;
        if ((P.unbounded & 8) && (int)cnt + 1 > P.max_dup) bad |= 8;
        nmsg += cnt ? 0 : 1;
    }
    if ((P.unbounded & 4) && nmsg > P.max_msgs) bad |= 4;
    return bad;
}

template <int S, int K>
RMC_HD Fp state_fp(const u64 (&w)[S], const u32 (&m)[K]) {
    Fp h{0, 0};
#pragma unroll
    for (int i = 0; i < S; ++i) fp_add(h, hS(w[i], (u32)i));
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (m[q]) fp_add(h, hM(m[q]));
    return h;
}

// Materialise a successor (only called for in-model successors) and put the
// bag in canonical order (descending, empty slots last).
template <int S, int K>
RMC_HD void materialise(const u64 (&w)[S], const u32 (&m)[K], const Delta& d, u64 (&wo)[S], u32 (&mo)[K]) {
#pragma unroll
    for (int i = 0; i < S; ++i) wo[i] = (d.srv == i) ? d.w_new : w[i];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        u32 sl = m[q];
        if (q == d.rm) sl = m_cnt(sl) > 1 ? sl - CNT_ONE : 0u;
        mo[q] = sl;
    }
    if (d.has_add) {
        int found = -1, hole = -1;
#pragma unroll
        for (int q = K - 1; q >= 0; --q) {
            found = (mo[q] && (mo[q] & MSG_MASK) == d.add) ? q : found;
            hole = mo[q] == 0 ? q : hole;
        }
#pragma unroll
        for (int q = 0; q < K; ++q) {
            if (q == found) mo[q] += CNT_ONE;
            else if (found < 0 && q == hole) mo[q] = d.add | CNT_ONE;
        }
    }
    // odd-even transposition sort, descending (K passes)
#pragma unroll
    for (int p = 0; p < K; ++p) {
#pragma unroll
        for (int q = (p & 1); q + 1 < K; q += 2) {
            const u32 a = mo[q], b = mo[q + 1];
            mo[q] = a > b ? a : b;
            mo[q + 1] = a > b ? b : a;
        }
    }
}

// ---- commuting diamonds: successors that need no probe ------------------------------
// Every stored state t remembers its first discoverer (parent s, lane a:
// t = a(s)); the footprint word below keeps the messages a acted on and
// added.  Expanding t, a successor b(t) is not probed when
//   (1) b precedes a in a fixed, state-independent order of action instances
//       (family, then the lane for server actions, the message for bag ones);
//   (2) a and b are independent: different server words (a lane reads and
//       writes at most one: Restart..AppendEntries their server i, Receive
//       the message's mdest, Duplicate/Drop none) and disjoint messages;
//   (3) b(s) satisfies the CONSTRAINT (only |DOMAIN messages| can differ from
//       b(t), by a's net change of the domain).
// Then b is enabled at s with the same effect and a(b(s)) = b(a(s)) = b(t):
// b(t) is generated from b(s), a state of the same or an earlier level, in
// the same or an earlier pass — and if a is skipped there too, the lane it
// relies on is later still in the order, so the chain ends.  Skipped
// successors still count as generated (TLC counts them); distinct counts,
// levels and depth are unchanged (tests/native/diamond_model.cpp checks it
// on whole BFS runs).  Not under SYMMETRY (canonical representatives break
// the instance order).
// Footprint word: bits 0-29 the message a acted on, 30-59 the message a added
// (both full 30-bit messages), 60-63 the flags below.  Every bit is taken.
constexpr u64 FOOT_VALID = 1ull << 63, FOOT_ACT = 1ull << 62, FOOT_ADD = 1ull << 61, FOOT_CONSUMED = 1ull << 60;
constexpr u64 FOOT_MSG_BITS = (u64)MSG_MASK | ((u64)MSG_MASK << 30);
static_assert((FOOT_MSG_BITS & (FOOT_VALID | FOOT_ACT | FOOT_ADD | FOOT_CONSUMED)) == 0,
              "footprint flags overlap the message fields");
// Sharded verification records only: the owner had seen this key (compare, do
// not store).  It lives in the record's global parent-ref word, whose bits
// 48-55 hold the rank (< kMaxWorld = 64) and 40-47 the lane: bit 63 is free.
constexpr u64 REF_SEEN = 1ull << 63;

// Family of a lane from the runtime offsets (wave-uniform lanes: scalar compares).
RMC_HD int lane_family(const Params& P, int lane) {
    int f = 0;
#pragma unroll
    for (int k = 1; k <= 9; ++k) f += lane >= P.off[k] ? 1 : 0;
    return f;
}
RMC_HD int family_off(const Params& P, int f) {
    int o = 0;
#pragma unroll
    for (int k = 0; k <= 9; ++k) o = f == k ? P.off[k] : o;
    return o;
}

// The footprint of t = lane(parent (w, m)) with delta d.
template <int S, int K>
RMC_HD u64 make_foot(const u32 (&m)[K], int lane, const Delta& d, const Params& P) {
    u64 f = FOOT_VALID;
    if (lane >= P.off[7]) {
        const int q = lane - (lane < P.off[8] ? P.off[7] : lane < P.off[9] ? P.off[8] : P.off[9]);
        f |= FOOT_ACT | (u64)(selm<K>(m, q) & MSG_MASK);
        if (d.rm >= 0) f |= FOOT_CONSUMED;
    }
    if (d.has_add) f |= FOOT_ADD | ((u64)(d.add & MSG_MASK) << 30);
    return f;
}

// make_foot from lane a's descriptor (no family-offset compares).
template <int S, int K>
RMC_HD u64 make_foot_desc(const u32 (&m)[K], u32 desc, const Delta& d) {
    u64 f = FOOT_VALID;
    if ((desc & 15u) >= 7u) {
        f |= FOOT_ACT | (u64)(selm<K>(m, (int)((desc >> 4) & 255u)) & MSG_MASK);
        if (d.rm >= 0) f |= FOOT_CONSUMED;
    }
    if (d.has_add) f |= FOOT_ADD | ((u64)(d.add & MSG_MASK) << 30);
    return f;
}

template <int S>
RMC_HD int lane_server(const Params& P, int lane, int fam, u32 msg) {
    const int t = lane - family_off(P, fam);
    return (fam == 0 || fam == 1 || fam == 3 || fam == 5) ? t
         : (fam == 2 || fam == 6) ? t / S
         : fam == 4 ? t / VMAX
         : fam == 7 ? (int)m_dst(msg) : -1;
}

template <int K>
RMC_HD int count_of(const u32 (&m)[K], u32 msg) {
    u32 c = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) c |= (m[q] && (m[q] & MSG_MASK) == msg) ? m_cnt(m[q]) : 0u;
    return (int)c;
}

// Per-lane descriptor (Params.ldesc): the family, the index inside it and the
// server whose word the lane's action writes (7: none, or the message's mdest
// for Receive) — what diamond_skip needs of lane b, read with one scalar load
// instead of recomputed from the family offsets in every lane of every state.
// Bits: family 0-3, index in the family 4-11, acting server 12-14 (7: none or
// per message), lane_delta_f's i 16-19 and j 20-23.
RMC_HD u32 lane_desc(const Params& P, int lane, int S) {
    const int f = lane_family(P, lane), t = lane - family_off(P, f);
    const int srv = (f == 0 || f == 1 || f == 3 || f == 5) ? t : (f == 2 || f == 6) ? t / S : f == 4 ? t / VMAX : 7;
    const int i = (f == 2 || f == 6) ? t / S : f == 4 ? t / VMAX : t;
    const int j = (f == 2 || f == 6) ? t % S : f == 4 ? t % VMAX : 0;
    return (u32)f | ((u32)t << 4) | ((u32)srv << 12) | ((u32)(i & 15) << 16) | ((u32)(j & 15) << 20);
}
RMC_HD void fill_lane_desc(Params& P, int S) {
    for (int l = 0; l < 128; ++l) P.ldesc[l] = l < P.off[10] ? lane_desc(P, l, S) : 0u;
}

// Per expanded state: a's side of the test (lane a = act, its footprint),
// packed into 4 words (it is live across the whole lane walk).
// Instance order key (0 = none): DropMessage instances first (by message), then
// the lanes of families 0-6 by (family, lane), then Receive and DuplicateMessage
// by (family, message): 1 + msg <= 2^30 < 2^30 + 1 + (f << 7 | lane) < 2^31 <=
// (f - 5) << 30 | msg (injective: every shape has fewer than 128 lanes).  Drop
// first: a Drop that commutes with the lane that discovered t is then skipped —
// 25.7 % fewer probes than with Drop last on MCraftBench's first 18 levels
// (tools/native/probe_classes.cpp), the same states.
RMC_HD u32 diamond_order(int f, int lane, u32 msg) {
    return f == 9 ? 1u + msg
         : f < 7 ? (1u << 30) + 1u + (((u32)f << 7) | (u32)lane)
                 : (((u32)(f - 5)) << 30) | msg;
}
struct Diamond {
    u32 ord;     // a's instance order key; 0 = no skipping from this state
    u32 k0, k1;  // a's messages (sentinels when absent; never equal to a 30-bit message)
    u32 sd;      // a's server word (bits 0-7, 0xFF none) | max |DOMAIN messages| of b(t) so that
                 // b(s) is in the model (bits 8-23) | DM_UNDO_ADD / DM_UNDO_DUP
};
// a added one copy of k1 and changed nothing else (RequestVote, AppendEntries,
// raft.tla:157-166, 171-192), or one copy of k0 (DuplicateMessage, :410-412):
// DropMessage of that message on t gives back a's parent s, a stored state
constexpr u32 DM_UNDO_ADD = 1u << 24, DM_UNDO_DUP = 1u << 25;
template <int S, int K>
RMC_HD void diamond_of(const u32 (&m)[K], int a, u64 foot, const Params& P, Diamond& dm) {
    dm.ord = 0;
    dm.k0 = 0xFFFFFFFFu;
    dm.k1 = 0xFFFFFFFEu;
    dm.sd = 0xFFu;
    if (a == 255 || !(foot & FOOT_VALID)) return;
    const int fa = lane_family(P, a);
    const u32 mact = (u32)(foot & MSG_MASK), madd = (u32)((foot >> 30) & MSG_MASK);
    dm.ord = diamond_order(fa, a, mact);
    if (foot & FOOT_ACT) dm.k0 = mact;
    if (foot & FOOT_ADD) dm.k1 = madd;
    const int srv = lane_server<S>(P, a, fa, mact);
    int delta = 0;
    if ((foot & FOOT_ADD) && count_of<K>(m, madd) == 1) delta += 1;       // a created the key
    if ((foot & FOOT_CONSUMED) && count_of<K>(m, mact) == 0) delta -= 1;  // a removed its last copy
    dm.sd = (u32)(srv & 0xFF) | ((u32)(P.max_msgs + delta) << 8);
    if ((fa == 2 || fa == 6) && (foot & FOOT_ADD)) dm.sd |= DM_UNDO_ADD;
    if (fa == 8 && (foot & FOOT_ACT)) dm.sd |= DM_UNDO_DUP;
}
RMC_HD bool diamond_rest(int sb, u32 mb, const Delta& db, int nmsg_b, const Diamond& dm) {
    if (sb >= 0 && (u32)sb == (dm.sd & 0xFFu)) return false;
    const u32 kb1 = db.has_add ? (db.add & MSG_MASK) : 0xFFFFFFFCu;
    if (mb == dm.k0 || mb == dm.k1 || kb1 == dm.k0 || kb1 == dm.k1) return false;
    return nmsg_b <= (int)((dm.sd >> 8) & 0xFFFFu);
}
// A shortcut checked before the order (it needs no diamond): b = DropMessage of
// the message a only added or duplicated (DM_UNDO_*) gives back s, a's parent.
// (A Receive that only removes its message has Drop's successor too — a "twin"
// rule skipping it measured slower for its extra registers: profiles/r05/samepar/.)
RMC_HD bool diamond_undo(int fb, u32 mb, const Diamond& dm) {
    return fb == 9 && ((mb == dm.k1 && (dm.sd & DM_UNDO_ADD)) || (mb == dm.k0 && (dm.sd & DM_UNDO_DUP)));
}
// b's side from lane b's descriptor: the same test as diamond_skip.
template <int S, int K>
RMC_HD bool diamond_skip_desc(const u32 (&m)[K], int b, u32 desc, const Delta& db, int nmsg_b, const Diamond& dm) {
    const int fb = (int)(desc & 15u), tb = (int)((desc >> 4) & 255u), sd = (int)((desc >> 12) & 7u);
    const u32 mb = fb >= 7 ? (selm<K>(m, tb) & MSG_MASK) : 0xFFFFFFFDu;
    if (diamond_undo(fb, mb, dm)) return true;
    if (!(diamond_order(fb, b, mb) < dm.ord)) return false;  // dm.ord = 0: never (the common exit)
    const int sb = sd < 7 ? sd : fb == 7 ? (int)m_dst(mb) : -1;
    return diamond_rest(sb, mb, db, nmsg_b, dm);
}
// b's side: lane b with delta db on t (m = t's bag), nmsg_b = |DOMAIN| of b(t).
template <int S, int K>
RMC_HD bool diamond_skip(const u32 (&m)[K], int b, const Delta& db, int nmsg_b, const Diamond& dm, const Params& P) {
    const int fb = lane_family(P, b);
    const u32 mb = fb >= 7 ? (selm<K>(m, b - family_off(P, fb)) & MSG_MASK) : 0xFFFFFFFDu;
    if (diamond_undo(fb, mb, dm)) return true;
    if (!(diamond_order(fb, b, mb) < dm.ord)) return false;  // dm.ord = 0: never
    return diamond_rest(lane_server<S>(P, b, fb, mb), mb, db, nmsg_b, dm);
}

// ---- invariants (fused into the insert of a new state) -----------------------------
template <int S, int K>
RMC_HD int type_ok(const u64 (&w)[S], const u32 (&m)[K], int V) {  // raft.tla:482-492
    for (int i = 0; i < S; ++i) {
        const u64 wi = w[i];
        if (w_st(wi) > LEADER) return 0;
        const u32 vf = w_vf(wi);
        if (vf != NILV && vf >= (u32)S) return 0;
        for (u32 x = 0; x < w_len(wi); ++x)
            if ((w_ent(wi, x) >> 4) >= (u32)V) return 0;
        // nextIndex >= 1 holds by construction (stored minus one)
    }
    for (int q = 0; q < K; ++q) {
        const u32 sl = m[q];
        if (!sl) continue;
        if (m_src(sl) >= (u32)S || m_dst(sl) >= (u32)S) return 0;
    }
    return 1;
}
template <int S>
RMC_HD int one_leader_per_term(const u64 (&w)[S]) {
    for (int i = 0; i < S; ++i)
        for (int j = i + 1; j < S; ++j)
            if (w_st(w[i]) == LEADER && w_st(w[j]) == LEADER && w_ct(w[i]) == w_ct(w[j])) return 0;
    return 1;
}
template <int S>
RMC_HD int log_matching(const u64 (&w)[S]) {  // raft.tla:1132-1136
    for (int i = 0; i < S; ++i)
        for (int j = i + 1; j < S; ++j) {
            const u32 li = w_len(w[i]), lj = w_len(w[j]);
            const u32 n = li < lj ? li : lj;
            for (u32 x = 1; x <= n; ++x) {
                if (ent_term(w_ent(w[i], x - 1)) != ent_term(w_ent(w[j], x - 1))) continue;
                const u64 pm = (1ull << (ENT_W * x)) - 1;
                if (((w[i] >> LOG_SH) & pm) != ((w[j] >> LOG_SH) & pm)) return 0;
            }
        }
    return 1;
}
// MessagesInv (raft.tla:941-946): every message in the bag satisfies
// RequestVoteResponseInv (:903-910, `m.dest` of :910 read as `m.mdest`),
// RequestVoteRequestInv (:915-920), AppendEntriesRequestInv (:924-930) and
// MessageTermsLtCurrentTerm (:934-935).  `log[src][mprevLogIndex + 1]` outside
// DOMAIN log[src] (a TLC evaluation error) counts as a violation.
template <int S, int K>
RMC_HD int messages_inv(const u64 (&w)[S], const u32 (&m)[K]) {
    for (int q = 0; q < K; ++q) {
        const u32 sl = m[q];
        if (!sl) continue;
        const u32 ty = m_type(sl), src = m_src(sl), dst = m_dst(sl), mt = m_term(sl);
        const u64 ws = selw<S>(w, (int)src), wd = selw<S>(w, (int)dst);
        const u32 cs = w_ct(ws);
        if (mt > cs) return 0;                                   // :934-935
        if (ty == RVP && ((sl >> 12) & 1u) && cs == w_ct(wd) && cs == mt) {  // :903-910
            const u32 ld = w_last_term(wd), ls = w_last_term(ws);
            if (!(ld > ls || (ld == ls && w_len(wd) >= w_len(ws)))) return 0;
        }
        if (ty == RVQ && w_st(ws) == CANDIDATE && cs == mt) {    // :915-920
            if (((sl >> 16) & 3u) != w_len(ws) || ((sl >> 12) & 15u) != w_last_term(ws)) return 0;
        }
        if (ty == AEQ && ((sl >> 19) & 1u) && mt == cs) {        // :924-930
            const u32 p1 = (sl >> 12) & 7u, n = w_len(ws);       // p1 = mprevLogIndex + 1
            if (p1 < 1 || p1 > n) return 0;                      // out of DOMAIN log[src]
            if (w_ent(ws, p1 - 1) != ((sl >> 20) & 31u)) return 0;
            if (p1 >= 2 && ent_term(w_ent(ws, p1 - 2)) != ((sl >> 15) & 15u)) return 0;
        }
    }
    return 1;
}
// LeaderVotesQuorum (raft.tla:1033-1037): a leader's term is backed by a quorum
// that voted for it or has moved to a higher term.
template <int S>
RMC_HD int leader_votes_quorum(const u64 (&w)[S]) {
    for (int i = 0; i < S; ++i) {
        if (w_st(w[i]) != LEADER) continue;
        const u32 ci = w_ct(w[i]);
        int n = 0;
        for (int j = 0; j < S; ++j)
            n += (w_ct(w[j]) > ci || (w_ct(w[j]) == ci && w_vf(w[j]) == (u32)i)) ? 1 : 0;
        if (2 * n <= S) return 0;
    }
    return 1;
}
// CandidateTermNotInLog (raft.tla:1041-1047): a candidate that can still win
// (a quorum of its term voted for it or not at all) has no entry of its term in
// any log.
template <int S>
RMC_HD int candidate_term_not_in_log(const u64 (&w)[S]) {
    for (int i = 0; i < S; ++i) {
        if (w_st(w[i]) != CANDIDATE) continue;
        const u32 ci = w_ct(w[i]);
        int n = 0;
        for (int j = 0; j < S; ++j) {
            const u32 vf = w_vf(w[j]);
            n += (w_ct(w[j]) == ci && (vf == (u32)i || vf == NILV)) ? 1 : 0;
        }
        if (2 * n <= S) continue;
        for (int j = 0; j < S; ++j)
            for (u32 x = 0; x < w_len(w[j]); ++x)
                if (ent_term(w_ent(w[j], x)) == ci) return 0;
    }
    return 1;
}
// The IsPrefix invariants (raft.tla:1143-1180) as restated in
// specs/MCraftBounded.tla: Committed(j) = the first min(commitIndex[j],
// Len(log[j])) entries of log[j].  IsPrefix(Committed(j), log[i]) compares
// packed entry bits.
RMC_HD int committed_prefix_of(u64 wj, u64 wi) {
    const u32 c = w_ci(wj) < w_len(wj) ? w_ci(wj) : w_len(wj);
    if (w_len(wi) < c) return 0;
    const u64 pm = (1ull << (ENT_W * c)) - 1;
    return ((wi >> LOG_SH) & pm) == ((wj >> LOG_SH) & pm);
}
template <int S>
RMC_HD int votes_granted_inv(const u64 (&w)[S]) {  // raft.tla:1145-1153
    for (int i = 0; i < S; ++i)
        for (int j = 0; j < S; ++j)
            if (((w_vg<S>(w[i]) >> j) & 1u) && w_ct(w[i]) == w_ct(w[j]) && !committed_prefix_of(w[j], w[i]))
                return 0;
    return 1;
}
template <int S>
RMC_HD int quorum_log_inv(const u64 (&w)[S]) {  // raft.tla:1157-1161
    for (int i = 0; i < S; ++i) {
        int miss = 0;  // servers lacking Committed(i): they must not contain a quorum
        for (int j = 0; j < S; ++j) miss += committed_prefix_of(w[i], w[j]) ? 0 : 1;
        if (2 * miss > S) return 0;
    }
    return 1;
}
template <int S>
RMC_HD int more_up_to_date_correct(const u64 (&w)[S]) {  // raft.tla:1167-1172
    for (int i = 0; i < S; ++i)
        for (int j = 0; j < S; ++j) {
            const u32 li = w_last_term(w[i]), lj = w_last_term(w[j]);
            if ((li > lj || (li == lj && w_len(w[i]) >= w_len(w[j]))) && !committed_prefix_of(w[j], w[i])) return 0;
        }
    return 1;
}
template <int S>
RMC_HD int leader_completeness(const u64 (&w)[S]) {  // raft.tla:1176-1180
    for (int i = 0; i < S; ++i) {
        if (w_st(w[i]) != LEADER) continue;
        for (int j = 0; j < S; ++j)
            if (!committed_prefix_of(w[j], w[i])) return 0;
    }
    return 1;
}
// The invariants other than TypeOK, out of line: inlined into every expansion
// kernel's new-state paths they would grow the code by ~15 % for checks that
// the bench model never names.  The state travels by value (in VGPRs).
template <int S, int K>
struct PackedState {
    u64 w[S];
    u32 m[K];
};
#if defined(__HIPCC__)
#define RMC_HD_COLD __host__ __device__ __noinline__
#else
#define RMC_HD_COLD inline
#endif
template <int S, int K>
RMC_HD_COLD int check_named_invariants(const PackedState<S, K> s, int mask) {
    if ((mask & 2) && !one_leader_per_term<S>(s.w)) return 2;
    if ((mask & 4) && !log_matching<S>(s.w)) return 3;
    if ((mask & 8) && !messages_inv<S, K>(s.w, s.m)) return 4;
    if ((mask & 16) && !leader_votes_quorum<S>(s.w)) return 5;
    if ((mask & 32) && !candidate_term_not_in_log<S>(s.w)) return 6;
    if ((mask & 64) && !votes_granted_inv<S>(s.w)) return 7;
    if ((mask & 128) && !quorum_log_inv<S>(s.w)) return 8;
    if ((mask & 256) && !more_up_to_date_correct<S>(s.w)) return 9;
    if ((mask & 512) && !leader_completeness<S>(s.w)) return 10;
    return 0;
}
// 0 = all hold, else 1 + index of the first violated invariant bit.
template <int S, int K>
RMC_HD int check_invariants(const u64 (&w)[S], const u32 (&m)[K], const Params& P) {
    if ((P.inv_mask & 1) && !type_ok<S, K>(w, m, P.V)) return 1;
    if (P.inv_mask & ~1) {
        PackedState<S, K> s;
        for (int i = 0; i < S; ++i) s.w[i] = w[i];
        for (int q = 0; q < K; ++q) s.m[q] = m[q];
        return check_named_invariants<S, K>(s, P.inv_mask);
    }
    return 0;
}

// ---- symmetry: server permutations -----------------------------------------------
// A permutation p (old server id -> new id, S <= 5) is packed 3 bits per
// entry into a u32 `code`, so applying it is shifts and masks: a small array
// indexed by runtime ids would be forced out of registers.
RMC_HD u32 pe(u32 code, u32 x) { return (code >> (3 * x)) & 7u; }
template <int S>
RMC_HD u64 perm_word(u64 w, u32 code) {  // the word moves to position pe(code, i)
    u64 r = w & (0x3Full | (0x3ull << CI_SH) | (0x1FFFFull << LEN_SH));  // ct, st, ci, log
    const u32 vf = w_vf(w);
    r |= (u64)(vf == NILV ? NILV : pe(code, vf)) << VF_SH;
#pragma unroll
    for (int j = 0; j < S; ++j) {
        const int pj = (int)pe(code, (u32)j);
        r |= ((w >> (SL<S>::VR + j)) & 1ull) << (SL<S>::VR + pj);
        r |= ((w >> (SL<S>::VG + j)) & 1ull) << (SL<S>::VG + pj);
        r |= ((w >> (SL<S>::NI + 2 * j)) & 3ull) << (SL<S>::NI + 2 * pj);
        r |= ((w >> (SL<S>::MI + 2 * j)) & 3ull) << (SL<S>::MI + 2 * pj);
    }
    return r;
}
RMC_HD u32 perm_slot(u32 sl, u32 code) {
    if (!sl) return 0;
    return (sl & ~(0xFCu)) | (pe(code, m_src(sl)) << 2) | (pe(code, m_dst(sl)) << 5);
}

// Canonical key under SYMMETRY Permutations(Server): the least fingerprint of
// the permuted states pi(s) over the permutations pi that SORT the servers by
// a permutation-invariant signature, every order of tied servers included.
// Relabelling s by sigma relabels the signatures the same way, so the set
// {pi(s)} -- and its least fingerprint -- is the same for every member of the
// orbit: an exact canonical key (up to fingerprint collisions), whatever the
// signature.  A weak signature only costs ties (more permutations to try);
// with messages folded in, 99 % of the MCraftBench states have none (measured
// on BFS levels 10-14), so a lane usually fingerprints ONE permuted state
// instead of all S! (DESIGN.md "SYMMETRY").
// Signature, part 1: the server word without server ids (term, role, commit
// index, log), votedFor as Nil / self / other, vote-set sizes and self bits,
// its own (nextIndex, matchIndex) and an order-free sum over its peers'.
template <int S>
RMC_HD u64 sig_base(u64 w, u32 i) {
    u64 s = w & (0x3Full | (0x7FFFFull << CI_SH));  // ct, st, ci, len, log
    const u32 vf = w_vf(w);
    s |= (u64)(vf == NILV ? 0u : vf == i ? 1u : 2u) << 6;
    const u32 vr = w_vr<S>(w), vg = w_vg<S>(w);
    s |= ((u64)__builtin_popcount(vr) << 28) | ((u64)__builtin_popcount(vg) << 31) |
         ((u64)((vr >> i) & 1u) << 34) | ((u64)((vg >> i) & 1u) << 35);
    u32 selfp = 0, others = 0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
        const u32 pr = (bits(w, SL<S>::NI + 2 * j, 2) << 2) | bits(w, SL<S>::MI + 2 * j, 2);
        if ((u32)j == i) selfp = pr;
        else others += (pr + 1u) * (pr + 7u);
    }
    return s | ((u64)selfp << 36) | ((u64)(others & 0xFFFFu) << 40);
}
// Signature, part 2: the messages a server sends and receives, ids masked,
// summed order-free.  Servers are ranked by (part 1, part 2) lexicographically:
// part 1 leads, so an action that only adds, duplicates or drops a message
// (RequestVote, AppendEntries, Duplicate, Drop: over half of the lanes) can
// reorder only servers whose part 1 ties.
RMC_HD u32 sig_src(u32 sl) { return (sl & ~0xFCu) * 0x9E3779B1u + 0x7F4A7C15u; }
RMC_HD u32 sig_dst(u32 sl) { return (sl & ~0xFCu) * 0x85EBCA77u + 0xC2B2AE3Du; }
template <int S>
struct Sig {
    u64 b[S];  // part 1 (sig_base)
    u32 m[S];  // part 2 (message sums)
};
template <int S, int K1>
RMC_HD void signatures(const u64 (&base)[S], const u32 (&m)[K1], Sig<S>& sg) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
        sg.b[i] = base[i];
        sg.m[i] = 0;
    }
#pragma unroll
    for (int q = 0; q < K1; ++q) {
        const u32 sl = m[q];
        const u32 a = sl ? sig_src(sl) : 0u, b = sl ? sig_dst(sl) : 0u;
        const u32 src = m_src(sl), dst = m_dst(sl);
#pragma unroll
        for (int i = 0; i < S; ++i) sg.m[i] += (src == (u32)i ? a : 0u) + (dst == (u32)i ? b : 0u);
    }
}
// Rank of every server by signature (3 bits each in *lo: server i -> its rank,
// the sorting permutation when nothing ties), the size of its tie class in
// *tc, and whether any two servers tie.
template <int S>
RMC_HD bool sig_rank(const Sig<S>& sg, u32* lo, u32* tc) {
    u32 l = 0, c = 0;
    bool tie = false;
#pragma unroll
    for (int i = 0; i < S; ++i) {
        u32 r = 0, n = 0;
#pragma unroll
        for (int j = 0; j < S; ++j) {
            const bool lt = sg.b[j] < sg.b[i] || (sg.b[j] == sg.b[i] && sg.m[j] < sg.m[i]);
            const bool eq = sg.b[j] == sg.b[i] && sg.m[j] == sg.m[i];
            r += lt ? 1u : 0u;
            n += eq ? 1u : 0u;
        }
        l |= r << (3 * i);
        c |= n << (3 * i);
        tie |= n > 1;
    }
    *lo = l;
    *tc = c;
    return tie;
}
// Fingerprint of pi(s) (any slot order; empty slots are 0).
template <int S, int K1>
RMC_HD Fp fp_perm(const u64 (&w)[S], const u32 (&m)[K1], u32 code) {
    Fp h{0, 0};
#pragma unroll
    for (int i = 0; i < S; ++i) fp_add(h, hS(perm_word<S>(w[i], code), pe(code, (u32)i)));
#pragma unroll
    for (int q = 0; q < K1; ++q)
        if (m[q]) fp_add(h, hM(perm_slot(m[q], code)));
    return h;
}
// The order of canonical candidates: least k, then least s.
RMC_HD bool fp_less(const Fp& a, const Fp& b) { return a.k < b.k || (a.k == b.k && a.s < b.s); }
// A state passed by value (out-of-line calls keep their registers apart).
template <int S, int K1>
struct SymState {
    u64 w[S];
    u32 m[K1];
};
// Ties (rare): the least fingerprint over every order of the tied servers,
// i.e. over the permutations whose position for server i lies in
// [lo_i, lo_i + tc_i) (3 bits per server in lo / tc).  Out of line: the
// common untied path stays small.
template <int S, int K1>
RMC_HD Fp canon_ties(const SymState<S, K1> t, u32 lo, u32 tc, const u32* codes, int np) {
    Fp best{~0ull, ~0u};
    for (int p = 0; p < np; ++p) {
        const u32 c = codes[p];
        bool ok = true;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            const u32 pos = pe(c, (u32)i), l = pe(lo, (u32)i);
            ok &= pos >= l && pos < l + pe(tc, (u32)i);
        }
        if (ok) {
            const Fp h = fp_perm<S, K1>(t.w, t.m, c);
            best = fp_less(h, best) ? h : best;
        }
    }
    return best;
}
// codes: every permutation of 0..S-1 (np = S!), for the tied case.  With
// NOTIE the tied case is not resolved here: *tied is set and 0 returned (the
// single-GPU SYMMETRY kernel defers those lanes to k_ties, so its hot loop
// carries no permutation enumeration).
template <int S, int K1, bool NOTIE = false>
RMC_HD Fp canon_sorted(const u64 (&w)[S], const u32 (&m)[K1], const Sig<S>& sg, const u32* codes, int np,
                       int* tied = nullptr) {
    u32 lo, tc;
    const bool tie = sig_rank<S>(sg, &lo, &tc);
    if (!tie) return fp_perm<S, K1>(w, m, lo);  // the sorting permutation: server i -> its rank
    if constexpr (NOTIE) {
        *tied = 1;
        return Fp{0, 0};
    }
    SymState<S, K1> t;
#pragma unroll
    for (int i = 0; i < S; ++i) t.w[i] = w[i];
#pragma unroll
    for (int q = 0; q < K1; ++q) t.m[q] = m[q];
    return canon_ties<S, K1>(t, lo, tc, codes, np);
}
// The canonical key of a stored (materialised) state.
template <int S, int K>
RMC_HD Fp canon_state(const u64 (&w)[S], const u32 (&m)[K], const u32* codes, int np) {
    u64 base[S];
#pragma unroll
    for (int i = 0; i < S; ++i) base[i] = sig_base<S>(w[i], (u32)i);
    Sig<S> sg;
    signatures<S, K>(base, m, sg);
    return canon_sorted<S, K>(w, m, sg, codes, np);
}
// The canonical key of the successor a delta makes of (w, m): the successor's
// words and slots (unsorted: fingerprints are order-free), the parent's
// signature bases reused for the servers the delta leaves alone.
template <int S, int K, bool NOTIE = false>
RMC_HD Fp canon_delta(const u64 (&w)[S], const u32 (&m)[K], const u64 (&base)[S], const Delta& d, const u32* codes,
                      int np, int* tied = nullptr) {
    u64 ws[S], bs[S];
    u32 ms[K + 1];
#pragma unroll
    for (int i = 0; i < S; ++i) {
        ws[i] = d.srv == i ? d.w_new : w[i];
        bs[i] = d.srv == i ? sig_base<S>(d.w_new, (u32)i) : base[i];
    }
    int found = -1;
#pragma unroll
    for (int q = 0; q < K; ++q) {
        u32 sl = m[q];
        if (q == d.rm) sl = m_cnt(sl) > 1 ? sl - CNT_ONE : 0u;
        ms[q] = sl;
        found = (d.has_add && sl && (sl & MSG_MASK) == d.add) ? q : found;
    }
    ms[K] = 0;
    if (d.has_add) {
#pragma unroll
        for (int q = 0; q < K; ++q) ms[q] += q == found ? CNT_ONE : 0u;
        ms[K] = found < 0 ? (d.add | CNT_ONE) : 0u;
    }
    Sig<S> sg;
    signatures<S, K + 1>(bs, ms, sg);
    return canon_sorted<S, K + 1, NOTIE>(ws, ms, sg, codes, np, tied);
}

}  // namespace rmc
