// rmc_kernels.hip — gfx950 kernels of the raft.tla BFS (DESIGN.md "Kernels").
//
//  k_expand : one lane per frontier state; loops over the state's action lanes
//             (Next raft.tla:421-430) in wave-uniform order, computes each
//             successor as a delta + incremental fingerprint, filters the
//             CONSTRAINT and stuttering successors, probes/CAS-inserts the
//             fingerprint into the HBM open-addressing set, and for the lanes
//             that won: wave-aggregated slot allocation, materialise, store,
//             parent pointer, fused invariant check.  Replaces TLC's worker
//             loop body (getNextStates + FPSet.put + invariant check).
//  k_seed   : inserts initial states (Init raft.tla:125-129) the same way.
//  k_list   : the same lane code with every enabled successor written out
//             (no dedup) — the differential-test entry point (rmc_expand).
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <map>
#include <mutex>

#include "raft_packed.h"
#include "rmc_internal.h"

namespace rmc {

__device__ __forceinline__ u64 bcast64(u64 v, int src) {
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)v, src);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), src);
    return ((u64)hi << 32) | lo;
}

// Open-addressing insert of a non-zero 64-bit value v whose probe sequence
// starts at slot s0, linear probing.
// Returns 1 if this lane inserted the key, 0 if it was present (or the table
// is full, flagged in *full).  Plain probe loads may be stale only in the
// EMPTY direction (slots go 0 -> key once); the CAS (agent scope, executed at
// the memory side) settles every race.
__device__ __forceinline__ int fp_insert(u64* __restrict__ table, u64 mask, u64 s0, u64 key, u32* full) {
    u64 s = s0;
    for (u64 n = 0; n <= mask; ++n) {
        const u64 cur = table[s];
        if (cur == key) return 0;
        if (fp_empty(cur)) {  // 0, or another epoch's entry (a tagged set)
            const u64 prev = atomicCAS((unsigned long long*)&table[s], (unsigned long long)cur, (unsigned long long)key);
            if (prev == cur) return 1;
            if (prev == key) return 0;
        }
        s = (s + 1) & mask;
    }
    atomicOr(full, 1u);
    return 0;
}

// fp_insert that also reports the slot holding the key (verification mode).
__device__ __forceinline__ int fp_insert_at(u64* __restrict__ table, u64 mask, u64 s0, u64 key, u32* full, u64* at) {
    u64 s = s0;
    for (u64 n = 0; n <= mask; ++n) {
        const u64 cur = table[s];
        if (cur == key) { *at = s; return 0; }
        if (fp_empty(cur)) {
            const u64 prev = atomicCAS((unsigned long long*)&table[s], (unsigned long long)cur, (unsigned long long)key);
            if (prev == cur) { *at = s; return 1; }
            if (prev == key) { *at = s; return 0; }
        }
        s = (s + 1) & mask;
    }
    atomicOr(full, 1u);
    *at = ~0ull;
    return 0;
}

// Same protocol, given the already-loaded content `cur` of the first slot s0.
__device__ __forceinline__ int fp_resolve(u64* __restrict__ table, u64 mask, u64 s0, u64 key, u64 cur, u32* full) {
    if (cur == key) return 0;
    if (fp_empty(cur)) {
        const u64 prev = atomicCAS((unsigned long long*)&table[s0], (unsigned long long)cur, (unsigned long long)key);
        if (prev == cur) return 1;
        if (prev == key) return 0;
    }
    return fp_insert(table, mask, s0, key, full);  // rare: continue linear probing
}
// Insert fingerprint h (raft_packed.h Fp) into the table.
__device__ __forceinline__ int fp_insert_fp(u64* __restrict__ table, u64 mask, const Fp& h, u32* full) {
    const TKey t = tkey(h, mask);
    return fp_insert(table, mask, t.s0, t.v, full);
}
// rmc_set_fp_bits (verification tests): only the kept bits of k, no second sum,
// so a weakened fingerprint collides as often as its width says.
__device__ __forceinline__ Fp fp_weaken(Fp h, u64 fp_mask) {
    if (fp_mask != ~0ull) {
        h.k &= fp_mask;
        h.s = 0;
    }
    return h;
}

template <int S, int K>
__device__ __forceinline__ void load_state(const u32* __restrict__ base, u64 (&w)[S], u32 (&m)[K]) {
    const u64* ws = reinterpret_cast<const u64*>(base);
#pragma unroll
    for (int i = 0; i < S; ++i) w[i] = ws[i];
    // Records are 8-byte aligned (2S + K words, K even), so the bag is read
    // as 8-byte pairs: a 16-byte load would be misaligned for odd S.
    if constexpr (K % 2 == 0) {
        const uint2* ms = reinterpret_cast<const uint2*>(base + 2 * S);
#pragma unroll
        for (int q = 0; q < K / 2; ++q) {
            const uint2 v = ms[q];
            m[2 * q] = v.x; m[2 * q + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int q = 0; q < K; ++q) m[q] = base[2 * S + q];
    }
}

template <int S, int K>
__device__ __forceinline__ void store_state(u32* __restrict__ base, const u64 (&w)[S], const u32 (&m)[K]) {
    u64* ws = reinterpret_cast<u64*>(base);
#pragma unroll
    for (int i = 0; i < S; ++i) ws[i] = w[i];
#pragma unroll
    for (int q = 0; q < K; ++q) base[2 * S + q] = m[q];
}

// Store one new state at index ni: the packed state, its trace link (global
// parent ref, lane), the footprint of its discovering lane (commuting
// diamonds; only shapes whose kernels skip diamonds keep them), its
// window-sort class (B.cls: a layout hint, read 1 B per state by the next
// level's window sort) and the fused invariant check.
template <int S, int K>
__device__ __forceinline__ void store_new(const Params& P, const DevBufs& B, u64 ni, const u64 (&wo)[S],
                                          const u32 (&mo)[K], u64 parent, int lane, u64 foot) {
    const u64 sl = wslot(B, ni);  // the ring window's slot (= ni unless spilling with links in HBM)
    store_state<S, K>(B.store + sl * (u64)(2 * S + K), wo, mo);
    B.parent[ni] = parent;
    B.act[ni] = (uint8_t)lane;
    B.foot[sl] = foot;
    B.cls[sl] = (uint8_t)state_class_fine<S, K>(wo, mo);
    const int v = check_invariants<S, K>(wo, mo, P);
    if (v) atomicMin((unsigned long long*)&B.ctr->viol, (unsigned long long)((ni << 4) | (u64)(v - 1)));
}

// Wave-aggregated allocation of store slots for the lanes with is_new set,
// then materialise + store + parent + invariants.  Must be reached by every
// lane of the wave (it contains a ballot).
template <int S, int K>
__device__ __forceinline__ void commit_new(int is_new, const u64 (&w)[S], const u32 (&m)[K], const Delta& d,
                                           const Params& P, const DevBufs& B, u64 parent_idx, int lane) {
    const u64 bal = __ballot(is_new);
    if (bal == 0) return;
    const int me = (int)__lane_id();
    const int leader = __ffsll((long long)bal) - 1;
    u64 base = 0;
    if (me == leader) base = atomicAdd((unsigned long long*)&B.ctr->count, (unsigned long long)__popcll(bal));
    base = bcast64(base, leader);
    if (!is_new) return;
    const u64 ni = base + (u64)__popcll(bal & ((1ull << me) - 1ull));
    if (ni >= B.cap) {
        atomicOr(&B.ctr->overflow, 1u);
        return;
    }
    u64 wo[S];
    u32 mo[K];
    materialise<S, K>(w, m, d, wo, mo);
    // initial states and deferred SYMMETRY ties: no diamond skipping from them
    store_new<S, K>(P, B, ni, wo, mo, parent_idx, lane, 0ull);
}

// Per-wave list of new states, kept in LDS until a flush materialises them.
constexpr int WCAP = 512;

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Replicated levels (sharded mode): one record per frontier state of the
// whole level, gathered from every rank — the packed state, its global ref
// (rank << 48 | index), its footprint and lane | class << 8 (k_pack_rep).
template <int S, int K>
struct RepRec {
    static constexpr int NW = 2 * S + K;
    static constexpr int REF = NW, FOOT = NW + 2, ACT = NW + 4;
    static constexpr int RR = NW + 6;  // words per record (8-byte aligned: NW is even)
};

// Materialise the wave's n listed new states: ONE global allocation atomic per
// flush, then each lane re-derives one listed successor from its parent
// (same lane_delta code, deterministic), stores it, its parent pointer and
// lane, and runs the fused invariant checks.  Convergent: the whole wave
// runs it together, so the rare new-state path does not serialise the
// per-lane expansion loop.  REP: the parents are replicated-level records
// (B.rep), their refs global.
template <int S, int K, bool REP = false>
__device__ __forceinline__ void flush_new(const Params& P, const DevBufs& B, u64 lo, const u32* l_rel,
                                          const uint8_t* l_lane, u32 n) {
    constexpr int NW = 2 * S + K;
    typedef RepRec<S, K> RR;
    wave_sync_lds();
    const int me = (int)__lane_id();
    u64 base = 0;
    if (me == 0) base = atomicAdd((unsigned long long*)&B.ctr->count, (unsigned long long)n);
    base = bcast64(base, 0);
    for (u32 e = (u32)me; e < n; e += 64) {
        const u64 rel = l_rel[e];
        const int lane = l_lane[e];
        const u64 ni = base + e;
        if (ni >= B.cap) {
            atomicOr(&B.ctr->overflow, 1u);
            continue;
        }
        u64 w[S];
        u32 m[K];
        const u32* pr = REP ? B.rep + (lo + rel) * (u64)RR::RR : B.store + wslot(B, lo + rel) * (u64)NW;
        load_state<S, K>(pr, w, m);
        Delta d;
        u64 foot;
        if constexpr (Lanes<S, K>::N <= 128) {  // the lane's descriptor: no family-offset compares
            const u32 desc = P.ldesc[lane];
            lane_delta_desc<S, K>(w, m, desc, P, d);
            foot = make_foot_desc<S, K>(m, desc, d);
        } else {
            lane_delta<S, K>(w, m, lane, P, d);
            foot = 0;
        }
        u64 wo[S];
        u32 mo[K];
        materialise<S, K>(w, m, d, wo, mo);
        const u64 parent = REP ? ((u64)pr[RR::REF] | ((u64)pr[RR::REF + 1] << 32)) : B.ref_tag | (lo + rel);
        store_new<S, K>(P, B, ni, wo, mo, parent, lane, foot);
    }
    wave_sync_lds();
}

__device__ __forceinline__ u64 wave_or64(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v |= (u64)(u32)__shfl_xor((int)(u32)v, off) | ((u64)(u32)__shfl_xor((int)(u32)(v >> 32), off) << 32);
    // the same on every lane: make it a scalar so the lane dispatch stays scalar branches
    const u32 lo = (u32)__builtin_amdgcn_readfirstlane((int)(u32)v);
    const u32 hi = (u32)__builtin_amdgcn_readfirstlane((int)(u32)(v >> 32));
    return ((u64)hi << 32) | lo;
}

// The OR over the wave's live states of lane_superset (raft_packed.h), built
// from one ballot per predicate instead of a shuffle reduction of the 64-bit
// masks: each bit of the mask is an OR of role / slot-occupancy predicates, so
// "some state of the wave has it" is a ballot.  Scalar result (SGPRs).
template <int S, int K>
__device__ __forceinline__ LaneMask lane_superset_wave(const u64 (&w)[S], const u32 (&m)[K], int V, bool live) {
    typedef Lanes<S, K> L;
    static_assert(L::N <= 128, "lane mask holds < 128 lanes");
    constexpr int O1 = L::off(1), O2 = L::off(2), O3 = L::off(3), O4 = L::off(4), O5 = L::off(5), O6 = L::off(6),
                  O7 = L::off(7), O8 = L::off(8), O9 = L::off(9);
    constexpr u64 SM = (1ull << S) - 1;
    LaneMask mk{0ull, 0ull};
    if (!__ballot(live)) return mk;
    mk.lo = SM;  // Restart(i): always enabled
#pragma unroll
    for (int i = 0; i < S; ++i) {
        const u32 st = w_st(w[i]);
        if (__ballot(live && st != LEADER)) mk.put(1ull, O1 + i);
        if (__ballot(live && st == CANDIDATE)) { mk.put(SM, O2 + i * S); mk.put(1ull, O3 + i); }
        if (__ballot(live && st == LEADER)) {
            mk.put((1ull << V) - 1, O4 + i * VMAX);
            mk.put(1ull, O5 + i);
            mk.put(SM, O6 + i * S);
        }
    }
#pragma unroll
    for (int q = 0; q < K; ++q)
        if (__ballot(live && m[q] != 0u)) { mk.put(1ull, O7 + q); mk.put(1ull, O8 + q); mk.put(1ull, O9 + q); }
    return mk;
}

// ---- full-state verification (RMC_FLAG_VERIFY_STATES) ---------------------------
// TLC trusts its 64-bit fingerprints; this mode checks them.  Every successor
// whose fingerprint is already in the set is compared, field for field, with
// the stored state that owns that fingerprint.  A difference is a fingerprint
// collision (a distinct state the search would silently drop) and is counted.
// The slot -> store-index map (sidx) is published between launches
// (k_publish), so a hit on a state of a completed launch is checked inline
// and a hit on a state found in the same launch is deferred to k_verify.
template <int S, int K>
__device__ __forceinline__ bool same_state(const u64 (&w)[S], const u32 (&m)[K], const u32* __restrict__ st) {
    u64 w2[S];
    u32 m2[K];
    load_state<S, K>(st, w2, m2);
    bool eq = true;
#pragma unroll
    for (int i = 0; i < S; ++i) eq &= w[i] == w2[i];
#pragma unroll
    for (int q = 0; q < K; ++q) eq &= m[q] == m2[q];
    return eq;
}

// SYMMETRY: the successor and the stored state are the same orbit iff some
// server permutation maps one onto the other (bag re-sorted after permuting).
template <int S, int K>
__device__ __noinline__ bool same_orbit(const PackedState<S, K> a, const u32* __restrict__ st, const PermTable& PT) {
    u64 w2[S];
    u32 m2[K];
    load_state<S, K>(st, w2, m2);
    for (int p = 0; p < PT.np; ++p) {
        const u32 c = PT.code[p];
        u64 wp[S];
        u32 mp[K];
#pragma unroll
        for (int t = 0; t < S; ++t) {
            u64 v = 0;
#pragma unroll
            for (int i = 0; i < S; ++i) v |= pe(c, (u32)i) == (u32)t ? perm_word<S>(a.w[i], c) : 0ull;
            wp[t] = v;
        }
#pragma unroll
        for (int q = 0; q < K; ++q) mp[q] = perm_slot(a.m[q], c);
#pragma unroll
        for (int r = 0; r < K; ++r) {
#pragma unroll
            for (int q = (r & 1); q + 1 < K; q += 2) {
                const u32 x = mp[q], y = mp[q + 1];
                mp[q] = x > y ? x : y;
                mp[q + 1] = x > y ? y : x;
            }
        }
        bool eq = true;
#pragma unroll
        for (int i = 0; i < S; ++i) eq &= wp[i] == w2[i];
#pragma unroll
        for (int q = 0; q < K; ++q) eq &= mp[q] == m2[q];
        if (eq) return true;
    }
    return false;
}

// Check one fingerprint hit: 0 = the stored state equals the successor,
// 1 = it differs (a collision), 2 = the owner is not published yet (defer),
// 3 = no slot (table full, flagged by the insert).  Counting and deferral are
// aggregated by the caller (one atomic per wave, not per hit).
template <int S, int K, bool SYM>
__device__ __forceinline__ int verify_hit(const u64 (&w)[S], const u32 (&m)[K], int lane, u64 slot, const Params& P,
                                       const PermTable& PT, const DevBufs& B) {
    constexpr int NW = 2 * S + K;
    if (slot == ~0ull) return 3;
    const u64 ix = B.sidx[slot];
    if (ix == ~0ull) return 2;  // owner found in this launch: check after it
    if (ix < B.vlo) return 4;   // owner spilled: checked against its host copy after the launch
    Delta d;
    lane_delta<S, K>(w, m, lane, P, d);
    PackedState<S, K> o;
    materialise<S, K>(w, m, d, o.w, o.m);
    const u32* st = B.store + wslot(B, ix) * (u64)NW;
    if constexpr (SYM) return same_orbit<S, K>(o, st, PT) ? 0 : 1;
    return same_state<S, K>(o.w, o.m, st) ? 0 : 1;
}

__device__ __forceinline__ u64 wave_sum64(u64 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v += (u64)(u32)__shfl_xor((int)(u32)v, off) | ((u64)(u32)__shfl_xor((int)(u32)(v >> 32), off) << 32);
    return v;
}

template <int S, int K, bool SYM>
__device__ __forceinline__ TKey verify_key(const u64 (&w)[S], const u32 (&m)[K], const Params& P, const PermTable& PT,
                                           u64 tmask) {
    return tkey(fp_weaken(SYM ? canon_state<S, K>(w, m, PT.code, PT.np) : state_fp<S, K>(w, m), P.fp_mask), tmask);
}

// sidx[slot of state i's fingerprint] = i for the stored states [lo, hi).
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_publish(const Params P, const PermTable PT, const DevBufs B, u64 lo, u64 hi) {
    constexpr int NW = 2 * S + K;
    for (u64 i = lo + (u64)blockIdx.x * 256ull + threadIdx.x; i < hi; i += (u64)gridDim.x * 256ull) {
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + wslot(B, i) * (u64)NW, w, m);
        const TKey key = verify_key<S, K, SYM>(w, m, P, PT, B.tmask);
        u64 s = key.s0;
        u64 n = 0;
        while (B.table[s] != key.v && n <= B.tmask) { s = (s + 1) & B.tmask; ++n; }
        if (n > B.tmask) atomicOr(&B.ctr->overflow, 8u);  // a stored state without its key
        else B.sidx[s] = i;
    }
}

// The deferred hits of the last launch, now that their owners are published.
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_verify(const Params P, const PermTable PT, const DevBufs B, u64 n) {
    constexpr int NW = 2 * S + K;
    u64 vchk = 0, vcol = 0;
    for (u64 q = (u64)blockIdx.x * 256ull + threadIdx.x; q < n; q += (u64)gridDim.x * 256ull) {
        const u64 parent = B.vbuf[2 * q], sl = B.vbuf[2 * q + 1];
        const u64 slot = sl & ((1ull << 56) - 1);
        const int lane = (int)(sl >> 56);
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + wslot(B, parent) * (u64)NW, w, m);
        Delta d;
        lane_delta<S, K>(w, m, lane, P, d);
        PackedState<S, K> o;
        materialise<S, K>(w, m, d, o.w, o.m);
        const u64 ix = B.sidx[slot];
        if (ix == ~0ull) {
            atomicOr(&B.ctr->overflow, 8u);
            continue;
        }
        ++vchk;
        const u32* st = B.store + wslot(B, ix) * (u64)NW;  // found in this launch: in the window
        bool same;
        if constexpr (SYM) same = same_orbit<S, K>(o, st, PT);
        else same = same_state<S, K>(o.w, o.m, st);
        vcol += same ? 0u : 1u;
    }
    vchk = wave_sum64(vchk);
    vcol = wave_sum64(vcol);
    if (__lane_id() == 0 && vchk) atomicAdd((unsigned long long*)&B.ctr->vchecked, (unsigned long long)vchk);
    if (__lane_id() == 0 && vcol) atomicAdd((unsigned long long*)&B.ctr->collisions, (unsigned long long)vcol);
}

// Verification + spill: the hits hbuf[off, off + n) whose owners had left the
// device window, against the owners' host copies staged at `owners` (one
// record each, in hbuf order).  The parents are the launch's frontier states,
// still in the window (the ring never overwrites a launch's own frontier).
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_verify_host(const Params P, const PermTable PT, const DevBufs B,
                                                     const u32* owners, u64 n, u64 off) {
    constexpr int NW = 2 * S + K;
    u64 vchk = 0, vcol = 0;
    for (u64 q = (u64)blockIdx.x * 256ull + threadIdx.x; q < n; q += (u64)gridDim.x * 256ull) {
        const u64 parent = B.hbuf[2 * (off + q)];
        const int lane = (int)(B.hbuf[2 * (off + q) + 1] >> 56);
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + wslot(B, parent) * (u64)NW, w, m);
        Delta d;
        lane_delta<S, K>(w, m, lane, P, d);
        PackedState<S, K> o;
        materialise<S, K>(w, m, d, o.w, o.m);
        const u32* st = owners + q * (u64)NW;
        bool same;
        if constexpr (SYM) same = same_orbit<S, K>(o, st, PT);
        else same = same_state<S, K>(o.w, o.m, st);
        ++vchk;
        vcol += same ? 0u : 1u;
    }
    vchk = wave_sum64(vchk);
    vcol = wave_sum64(vcol);
    if (__lane_id() == 0 && vchk) atomicAdd((unsigned long long*)&B.ctr->vchecked, (unsigned long long)vchk);
    if (__lane_id() == 0 && vcol) atomicAdd((unsigned long long*)&B.ctr->collisions, (unsigned long long)vcol);
}

// Owner rank of a state in sharded mode.  Mode 0: by fingerprint.  Mode 1: by
// server 0's word — a successor that does not touch server 0 (bag-only
// actions, actions of the other servers) stays on its parent's rank, so far
// fewer successors cross GPUs; balance relies on server 0's many word values.
// Mode 2 (default): by the words of servers 0 and 1 (more distinct values:
// better balance, successors of two servers cross).  The word hash is the
// fingerprint's own component mix hS(w, i): the expansion kernel has the
// parent's mixes and the new word's mix at hand, so routing a successor costs
// no extra mix64 (and no extra registers) in its lane loop.
// Number of server words the owner hashes: mode 1 one, 2 two, 3 all S.
template <int S>
__device__ __forceinline__ int owner_words(const DevBufs& B) {
    return B.owner_mode >= 3 ? S : (int)B.owner_mode;
}
template <int S>
__device__ __forceinline__ u32 owner_state(u64 key, const u64 (&w)[S], const DevBufs& B) {
    if (B.owner_mode == 0) return owner_of(key, B.world);
    const int nw = owner_words<S>(B);
    u64 h = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) h += i < nw ? hS(w[i], (u32)i) : 0ull;
    return owner_of(h, B.world);
}
// Owner of a successor from the parent's words (kernels without the parent's mixes).
template <int S>
__device__ __forceinline__ u32 owner_succ_w(u64 key, const Delta& d, const u64 (&w)[S], const DevBufs& B) {
    if (B.owner_mode == 0) return owner_of(key, B.world);
    if (d.srv < 0 || d.srv >= owner_words<S>(B)) return B.rank;
    u64 ws[S];
#pragma unroll
    for (int i = 0; i < S; ++i) ws[i] = i == d.srv ? d.w_new : w[i];
    return owner_state<S>(key, ws, B);
}
// Owner of a successor from the parent's word mixes (pm.hw) and the new word's
// mix hn (delta_fp_pre): a lane that leaves the hashed words alone keeps its
// parent's owner `powner` — this rank in the sharded kernel (a state is
// expanded by its owner), the record's rank in a replicated level.
template <int S, int K>
__device__ __forceinline__ u32 owner_succ(u64 key, const Delta& d, const ParentMix<S, K>& pm, u64 hn,
                                          const DevBufs& B, u32 powner) {
    if (B.world == 1) return 0;
    if (B.owner_mode == 0) return owner_of(key, B.world);
    const int nw = owner_words<S>(B);
    if (d.srv < 0 || d.srv >= nw) return powner;
    u64 h = 0;
#pragma unroll
    for (int i = 0; i < S; ++i) h += i < nw ? (i == d.srv ? hn : pm.hw[i]) : 0ull;
    return owner_of(h, B.world);
}

template <int S, int K>
__device__ __forceinline__ Fp fp_of_materialised(const u64 (&w)[S], const u32 (&m)[K], const Params& P) {
    return state_fp<S, K>(w, m);  // = the incremental key: the fp is order-free
}

// Phase-1 keys travel as the raw fingerprint (k, low 32 bits of s): the owner
// derives its own table value and slot (tkey; tables may differ in size across
// ranks).  Outbox: 12 B per key, three u32 {k lo, k hi, s32} (round 6; 16 B
// before: a quarter of phase 1's bytes was padding); parking (B.ovf): {k, s32 | flags << 32,
// ticket}, where flag OVF_UNKEYED marks a ticket the expansion parked without
// computing its key (k_route_fix computes it).
constexpr u64 OVF_UNKEYED = 1ull << 32;
__device__ __forceinline__ void put_key(const DevBufs& B, u32 dest, u64 slot, u64 k, u32 s32, u64 tick) {
    u32* o = reinterpret_cast<u32*>(B.key_out) + 3 * ((u64)dest * B.kcap + slot);
    o[0] = (u32)k;
    o[1] = (u32)(k >> 32);
    o[2] = s32;
    B.tick_out[(u64)dest * B.kcap + slot] = tick;
}
__device__ __forceinline__ void park_key(const DevBufs& B, u64 k, u64 s_and_flags, u64 tick) {
    const u64 q = atomicAdd((unsigned long long*)&B.ctr->novf, 1ull);
    if (q < B.ovf_cap) {
        B.ovf[3 * q] = k;
        B.ovf[3 * q + 1] = s_and_flags;
        B.ovf[3 * q + 2] = tick;
    } else {
        atomicOr(&B.ctr->overflow, 2u);  // the parking buffer is full too: fatal
    }
}

// Sharded mode, phase 1 (fingerprint first): the listed
// successors carry their owner rank.  Owned ones were inserted into the local
// set at probe time and are stored as in flush_new; for the others only the
// key travels: it goes to the owner's key outbox, with a local ticket (parent
// index | lane << 56) kept here so that, if the owner answers "new", phase 2
// re-derives the successor and ships the state.  Slots are reserved with one
// atomic per destination per flush.
template <int S, int K>
__device__ __forceinline__ void flush_dist(const Params& P, const DevBufs& B, u64 lo, const u32* l_rel,
                                           const uint8_t* l_lane, const uint8_t* l_dest, const u64* l_key,
                                           const u32* l_ks, u32 n) {
    constexpr int NW = 2 * S + K;
    wave_sync_lds();
    const int me = (int)__lane_id();
    const u64 lt = (1ull << me) - 1ull;
    // Reserve every destination's slots for the whole list with ONE atomic per
    // destination: lane dd (world <= 64) counts destination dd's entries, adds
    // them to dd's counter, then hands out consecutive slots round by round.
    u64 mine = 0;  // lane dd: entries for destination dd, then its next slot
    for (u32 e0 = 0; e0 < n; e0 += 64) {
        const u32 e = e0 + (u32)me;
        const u32 dest = e < n ? l_dest[e] : 0xFFu;
        for (u32 dd = 0; dd < B.world; ++dd) {
            const u64 bal = __ballot(dest == dd);
            if ((u32)me == dd) mine += (u64)__popcll(bal);
        }
    }
    if ((u32)me < B.world && mine) {
        unsigned long long* ctr = (u32)me == B.rank ? (unsigned long long*)&B.ctr->count : &B.ocount[me];
        mine = atomicAdd(ctr, (unsigned long long)mine);
    }
    for (u32 e0 = 0; e0 < n; e0 += 64) {  // wave-uniform rounds
        const u32 e = e0 + (u32)me;
        const bool valid = e < n;
        const u32 dest = valid ? l_dest[e] : 0xFFu;
        u64 slot = ~0ull;
        for (u32 dd = 0; dd < B.world; ++dd) {
            const u64 bal = __ballot(dest == dd);
            if (!bal) continue;
            const u64 base = bcast64(mine, (int)dd);
            if (dest == dd) slot = base + (u64)__popcll(bal & lt);
            if ((u32)me == dd) mine += (u64)__popcll(bal);
        }
        if (!valid) continue;
        const u64 rel = l_rel[e];
        const int lane = l_lane[e];
        if (dest != B.rank) {  // the key to its owner, the ticket stays here
            if (slot >= B.kcap) {
                // the owner's outbox is full: park the key with its ticket; a later
                // exchange round of this level sends it (the sent-cache entry
                // written at probe time stays right: the key IS sent)
                // (the list holds the local table value: the raw k is v ^ (s32 & tmask))
                park_key(B, l_key[e] ^ ((u64)l_ks[e] & B.tmask), l_ks[e],
                         (lo + rel) | ((u64)dest << 48) | ((u64)lane << 56));
                continue;
            }
            put_key(B, dest, slot, l_key[e] ^ ((u64)l_ks[e] & B.tmask), l_ks[e], (lo + rel) | ((u64)lane << 56));
            continue;
        }
        if (slot >= B.cap) {
            atomicOr(&B.ctr->overflow, 1u);
            continue;
        }
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + (lo + rel) * (u64)NW, w, m);
        Delta d;
        lane_delta<S, K>(w, m, lane, P, d);
        u64 wo[S];
        u32 mo[K];
        materialise<S, K>(w, m, d, wo, mo);
        store_new<S, K>(P, B, slot, wo, mo, B.ref_tag | (lo + rel), lane, make_foot<S, K>(m, lane, d, P));
    }
    wave_sync_lds();
}

// Sharded mode with send markers (MARK): the local fingerprint set doubles
// as the record of keys already sent — a successor owned elsewhere is
// CAS-inserted into it like a local one, so the probe loop is the single-GPU
// loop (no owner computed per probe) and a remote key is shipped at most once
// per rank (a lossless sent-cache).  The list carries only (rel, lane); here
// each listed successor's owner is found from its changed word (a first pass,
// only with more than one rank, into l_dest), then each is re-derived: owned
// ones are stored as in
// flush_new, the others get their key back from the materialised successor
// (the fingerprint is order-free: it equals the incremental probe key) and go
// to the owner's outbox with a ticket.  One reservation atomic per destination.
template <int S, int K>
__device__ __forceinline__ void flush_mark(const Params& P, const DevBufs& B, u64 lo, const u32* l_rel,
                                           const uint8_t* l_lane, uint8_t* l_dest, u32 n) {
    constexpr int NW = 2 * S + K;
    wave_sync_lds();
    const int me = (int)__lane_id();
    const u64 lt = (1ull << me) - 1ull;
    u64 mine = 0;  // lane dd: entries for destination dd, then its next slot
    for (u32 e0 = 0; e0 < n; e0 += 64) {
        const u32 e = e0 + (u32)me;
        u32 dest = 0xFFu;
        if (e < n) {
            dest = 0;
            if (B.world > 1) {
                u64 w[S];
                u32 m[K];
                load_state<S, K>(B.store + (lo + l_rel[e]) * (u64)NW, w, m);
                Delta d;
                if constexpr (Lanes<S, K>::N <= 128) lane_delta_desc<S, K>(w, m, P.ldesc[l_lane[e]], P, d);
                else lane_delta<S, K>(w, m, l_lane[e], P, d);
                if (B.owner_mode == 0) {
                    u64 wo[S];
                    u32 mo[K];
                    materialise<S, K>(w, m, d, wo, mo);
                    dest = owner_of(fp_of_materialised<S, K>(wo, mo, P).k, B.world);
                } else {
                    dest = owner_succ_w<S>(0ull, d, w, B);
                }
                l_dest[e] = (uint8_t)dest;
            }
        }
        for (u32 dd = 0; dd < B.world; ++dd) {
            const u64 bal = __ballot(dest == dd);
            if ((u32)me == dd) mine += (u64)__popcll(bal);
        }
    }
    if ((u32)me < B.world && mine) {
        unsigned long long* ctr = (u32)me == B.rank ? (unsigned long long*)&B.ctr->count : &B.ocount[me];
        mine = atomicAdd(ctr, (unsigned long long)mine);
    }
    for (u32 e0 = 0; e0 < n; e0 += 64) {  // wave-uniform rounds
        const u32 e = e0 + (u32)me;
        const bool valid = e < n;
        const u32 dest = !valid ? 0xFFu : B.world > 1 ? (u32)l_dest[e] : 0u;
        u64 slot = ~0ull;
        for (u32 dd = 0; dd < B.world; ++dd) {
            const u64 bal = __ballot(dest == dd);
            if (!bal) continue;
            const u64 base = bcast64(mine, (int)dd);
            if (dest == dd) slot = base + (u64)__popcll(bal & lt);
            if ((u32)me == dd) mine += (u64)__popcll(bal);
        }
        if (!valid) continue;
        const u64 rel = l_rel[e];
        const int lane = l_lane[e];
        if (dest == B.rank && slot >= B.cap) {
            atomicOr(&B.ctr->overflow, 1u);
            continue;
        }
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + (lo + rel) * (u64)NW, w, m);
        Delta d;
        u64 foot;
        if constexpr (Lanes<S, K>::N <= 128) {  // the lane's descriptor: no family-offset compares
            const u32 desc = P.ldesc[lane];
            lane_delta_desc<S, K>(w, m, desc, P, d);
            foot = make_foot_desc<S, K>(m, desc, d);
        } else {
            lane_delta<S, K>(w, m, lane, P, d);
            foot = 0;
        }
        u64 wo[S];
        u32 mo[K];
        materialise<S, K>(w, m, d, wo, mo);
        if (dest != B.rank) {  // the key to its owner, the ticket stays here
            const Fp key = fp_of_materialised<S, K>(wo, mo, P);
            if (slot >= B.kcap) {  // outbox full: parked, sent by a later round of this level
                park_key(B, key.k, (u32)key.s, (lo + rel) | ((u64)dest << 48) | ((u64)lane << 56));
                continue;
            }
            put_key(B, dest, slot, key.k, (u32)key.s, (lo + rel) | ((u64)lane << 56));
            continue;
        }
        store_new<S, K>(P, B, slot, wo, mo, B.ref_tag | (lo + rel), lane, foot);
    }
    wave_sync_lds();
}

// Sharded mode with send markers, the pool flush (default): flush_new with the
// owner decided per listed successor from its materialised words — a lane that
// leaves the hashed words alone keeps its parent's owner, this rank — and two
// reservation atomics per 64 entries, one for the local store, one for the
// remote-successor pool (B.pool).  A remote successor is written there once, as
// its phase-2 record; keying it, the per-destination slots and parking are left
// to k_route after the launch.  So the flush carries no per-destination
// bookkeeping, no second pass over the list and no re-hash of the successor,
// and the sharded kernel keeps the single-GPU kernel's registers.  A pool that
// is full parks the successor's ticket with key 0 (k_route keys it).
template <int S, int K>
__device__ __forceinline__ void flush_pool(const Params& P, const DevBufs& B, u64 lo, const u32* l_rel,
                                           const uint8_t* l_lane, uint8_t* l_own, u32 n) {
    constexpr int NW = 2 * S + K, RW = NW + 4;
    wave_sync_lds();
    const int me = (int)__lane_id();
    const u64 lt = (1ull << me) - 1ull;
    // pass 1 (more than one rank): which listed successors this rank owns (LDS
    // byte per entry): only lanes that change a hashed server word can leave
    u32 nown = n;  // wave-uniform
    if (B.world > 1) {
        nown = 0;
        for (u32 e0 = 0; e0 < n; e0 += 64) {
            const u32 e = e0 + (u32)me;
            bool own = true;
            if (e < n) {
                const int lane = l_lane[e];
                Delta d;
                u64 w[S];
                u32 m[K];
                load_state<S, K>(B.store + (lo + l_rel[e]) * (u64)NW, w, m);
                if constexpr (Lanes<S, K>::N <= 128) lane_delta_desc<S, K>(w, m, P.ldesc[lane], P, d);
                else lane_delta<S, K>(w, m, lane, P, d);
                if (B.owner_mode == 0) {
                    u64 wo[S];
                    u32 mo[K];
                    materialise<S, K>(w, m, d, wo, mo);
                    own = owner_of(fp_of_materialised<S, K>(wo, mo, P).k, B.world) == B.rank;
                } else if (d.srv >= 0 && d.srv < owner_words<S>(B)) {
                    own = owner_succ_w<S>(0ull, d, w, B) == B.rank;
                }
                l_own[e] = own ? 1 : 0;
            }
            nown += (u32)__popcll(__ballot(e < n && own));
        }
        wave_sync_lds();
    }
    u64 base_l = 0, base_r = 0;
    if (me == 0 && nown) base_l = atomicAdd((unsigned long long*)&B.ctr->count, (unsigned long long)nown);
    if (me == 0 && n > nown) base_r = atomicAdd(B.npool, (unsigned long long)(n - nown));
    base_l = bcast64(base_l, 0);
    base_r = bcast64(base_r, 0);
    for (u32 e0 = 0; e0 < n; e0 += 64) {  // wave-uniform rounds
        const u32 e = e0 + (u32)me;
        const bool valid = e < n;
        const bool own = valid && (B.world == 1 || l_own[e]);
        const u64 bl = __ballot(own), br = __ballot(valid && !own);
        const u64 ql = base_l + (u64)__popcll(bl & lt), qr = base_r + (u64)__popcll(br & lt);
        base_l += (u64)__popcll(bl);
        base_r += (u64)__popcll(br);
        if (!valid) continue;
        const u64 rel = l_rel[e];
        const int lane = l_lane[e];
        if (own && ql >= B.cap) {
            atomicOr(&B.ctr->overflow, 1u);
            continue;
        }
        if (!own && qr >= B.pool_cap) {  // pool full: park the ticket, k_route_fix keys it
            park_key(B, 0ull, OVF_UNKEYED, (lo + rel) | ((u64)lane << 56));
            continue;
        }
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + (lo + rel) * (u64)NW, w, m);
        Delta d;
        u64 foot;
        if constexpr (Lanes<S, K>::N <= 128) {
            const u32 desc = P.ldesc[lane];
            lane_delta_desc<S, K>(w, m, desc, P, d);
            foot = make_foot_desc<S, K>(m, desc, d);
        } else {
            lane_delta<S, K>(w, m, lane, P, d);
            foot = make_foot<S, K>(m, lane, d, P);
        }
        u64 wo[S];
        u32 mo[K];
        materialise<S, K>(w, m, d, wo, mo);
        const u64 parent = B.ref_tag | (lo + rel);
        if (own) {
            store_new<S, K>(P, B, ql, wo, mo, parent, lane, foot);
            continue;
        }
        u32* r = B.pool + qr * (u64)RW;
        store_state<S, K>(r, wo, mo);
        const u64 ref = parent | ((u64)lane << 40);
        r[NW] = (u32)ref;
        r[NW + 1] = (u32)(ref >> 32);
        r[NW + 2] = (u32)foot;
        r[NW + 3] = (u32)(foot >> 32);
    }
    wave_sync_lds();
}

// Grid-stride over 256-state tiles of the frontier [lo, hi).  Lanes are
// processed BATCH at a time so BATCH fingerprint probes per thread are in
// flight together (the kernel is bound by probe latency, not bandwidth).
// SORT: the lane-superset walk — each block takes windows of WTILES tiles and
//   walks their states in class order (a counting sort in LDS over the 1-byte
//   classes B.cls), so its waves hold states of one kind and walk only the
//   lanes some state of the wave can enable (lane_superset, a scalar).
// DIST: sharded mode — successors owned by another rank go to that owner's
//   key outbox: with MARK (the default) after a CAS into the local set (send
//   markers: a lossless sent-cache), else through the lossy sent-cache B.sent
//   (SYMMETRY and verification).
// DIA: commuting-diamond successors are not probed (raft_packed.h "commuting
//   diamonds"; P.diamond = 0 turns it off at run time).
// PIPE: a probe's load is issued as soon as its key is known, so the loads
//   overlap the lane code of the batch's later lanes (266-272 vs 271-279 ms
//   per bench BFS, profiles/r03/ab/probe_issue_r03pipe*.jsonl).
// REP: a replicated level of the sharded search — [lo, hi) indexes the whole
//   level's records in B.rep (gathered from every rank); every rank expands
//   all of them and probes, stores and counts only the successors it owns.
template <int S, int K, bool SYM, int BATCH, bool DIST, bool VERIFY = false, bool PRE = false, bool SORT = false,
          bool DIA = false, bool MARK = false, int WTILES = 8, int PIPE = 0, bool REP = false, bool PRESORT = false,
          int DYN = 0, bool POOL = false>
__device__ __forceinline__ void expand_body(const Params& P, const PermTable& PT, const DevBufs& B, u64 lo, u64 hi) {
    static_assert(!MARK || (DIST && !VERIFY && !SYM), "send markers: the plain sharded kernel only");
    static_assert(!POOL || (MARK && !REP), "the pool flush: the send-marker kernel");
    constexpr bool SENTC = DIST && !MARK;  // the lossy sent-cache + (key, dest) list entries
    static_assert(!DIA || (!SYM && !VERIFY), "diamond skipping: not under SYMMETRY or verification");
    static_assert(!SORT || !VERIFY, "SORT: not with verification");
    static_assert(!SORT || BATCH * 7 <= 64, "SORT packs a batch's lanes 7 bits each into one u64");
    static_assert(PIPE == 0 || (!SYM && !VERIFY && !SENTC), "PIPE: the plain and marker kernels");
    static_assert(!REP || (MARK && SORT && PRE), "replicated levels: the plain sharded kernel");
    // PRESORT: the windows were counting-sorted by class before the launch
    // (k_window_order writes each window's positions in class order to B.word),
    // so the kernel carries no sort: no LDS bins, scan or block barriers
    static_assert(!PRESORT || (SORT && !REP), "presorted windows: the sorted kernels");
    constexpr bool INSORT = SORT && !PRESORT;
    // DYN: each wave takes its next unit of work — one wave's quarter of a
    // presorted window (its 64 lanes of every tile) — from a launch-wide
    // counter, instead of the block's fixed share of windows: the waves end
    // together however unequal the units' costs and whatever the window count
    static_assert(DYN == 0 || PRESORT, "dynamic units: presorted windows");
    // (the marker kernel measured no gain from PIPE at one rank: 308.7-309.7 vs 307.4-308.7 ms)
    constexpr int NW = 2 * S + K;
    typedef RepRec<S, K> RR;
    constexpr int FW = REP ? RR::RR : NW;  // words per frontier record
    const u32* const fr = REP ? B.rep : B.store;
    constexpr bool TIEDEFER = SYM && !DIST && !VERIFY;
    constexpr bool LISTOWN = SENTC;  // list entries carry their owner (MARK: found at flush time)
    constexpr int WT = SORT ? WTILES : 1;   // tiles per window
    __shared__ uint16_t s_ord[INSORT ? 256 * WT : 1];  // window positions in class order
    __shared__ uint8_t s_wcls[INSORT ? 256 * WT : 1];  // class of each window position
    constexpr int NBIN = 256;                           // roles x message-count classes
    __shared__ u32 s_wbin[INSORT ? NBIN : 1];           // class counters / cursors
    // Sharded mode keeps per-probe owners in LDS too; a shorter list keeps the
    // block under 160 KB / 6 so it runs at the same 6 waves/SIMD as the
    // single-GPU kernel (VGPR-bound there).
    constexpr int LCAP = SENTC ? 256 : MARK ? WCAP - 64 : WCAP;  // MARK: the owner byte per entry
    __shared__ u32 s_rel[4][LCAP];
    __shared__ uint8_t s_lane[4][LCAP];
    constexpr bool LDEST = SENTC || MARK;
    __shared__ uint8_t s_dest[LDEST ? 4 : 1][LDEST ? LCAP : 1];  // owner per listed successor
    __shared__ u64 s_lkey[SENTC ? 4 : 1][SENTC ? LCAP : 1];  // sharded: the key of each listed successor
    __shared__ u32 s_lks[SENTC ? 4 : 1][SENTC ? LCAP : 1];   // ... and its s32 (fp_norm)
    __shared__ u64 s_key[BATCH][256];  // per lane of the batch: the probe's table value (0 = no probe)
    __shared__ u32 s_ks[BATCH][256];   // ... and its s32, which recovers its slot (fp_slot)
    __shared__ uint8_t s_own[LISTOWN ? BATCH : 1][LISTOWN ? 256 : 1];  // owner rank per probe
    const int wv = (int)(threadIdx.x >> 6);
    const int me = (int)__lane_id();
    const u64 lt_mask = (1ull << me) - 1ull;
    u32* l_rel = s_rel[wv];
    uint8_t* l_lane = s_lane[wv];
    uint8_t* l_dest = s_dest[LDEST ? wv : 0];
    u64* l_key = s_lkey[SENTC ? wv : 0];
    u32* l_ks = s_lks[SENTC ? wv : 0];
    u32 n = 0;  // wave-uniform list length
    u32 gen = 0;  // generated lanes of this thread's states (< 2^32 per launch)
    u64 vchk = 0, vcol = 0;  // verification: hits compared, collisions
    u64 pr = 0;  // probes issued by the whole wave (wave-uniform)
    u32 walked = 0;  // (live state, lane) slots this thread's waves visited for it
    const u64 nf = hi - lo;
    const int nl = P.off[10];  // == Lanes<S,K>::N; runtime on purpose (see lane_delta)
    // tiles per window, fewer when the launch has too few states to give every
    // block a full window (small levels would idle most blocks)
    u64 wt = WT;
    if constexpr (SORT) {
        const u64 per_block = (nf + (u64)gridDim.x * 256ull - 1) / ((u64)gridDim.x * 256ull);
        wt = per_block < (u64)WT ? (per_block ? per_block : 1ull) : (u64)WT;
    }
    u32 q64 = (u32)threadIdx.x & ~63u;  // this thread's window slot base (DYN: the unit's)
    u64 win = DYN ? 0ull : (u64)blockIdx.x * 256ull * wt;
    for (;; win += (u64)gridDim.x * 256ull * wt) {  // block-uniform (DYN: wave-uniform)
    if constexpr (DYN != 0) {
        u32 unit = 0;
        if (me == 0) unit = (u32)atomicAdd((unsigned long long*)&B.ctr->wnext, 1ull);
        unit = (u32)__builtin_amdgcn_readfirstlane(__shfl((int)unit, 0));
        win = (u64)(unit >> 2) * 256ull * wt;
        q64 = (unit & 3u) * 64u;
    }
    if (win >= nf) break;
    u32 wn = 0;  // SORT: states in this window
    if constexpr (SORT) wn = (u32)((nf - win) < 256ull * wt ? (nf - win) : 256ull * wt);
    if constexpr (INSORT) {
        __syncthreads();  // the previous window's s_ord is consumed
        if (threadIdx.x < NBIN) s_wbin[threadIdx.x] = 0;
        __syncthreads();
        for (int k = 0; k < (int)wt; ++k) {
            const u32 p = (u32)k * 256u + threadIdx.x;
            if (p < wn) {
                // the stored 1-byte class (B.cls / the record's class byte), not the state
                const u32 c = REP ? (fr[(lo + win + p) * (u64)FW + RR::ACT] >> 8) & 0xFFu
                                  : (u32)B.cls[wslot(B, lo + win + p)];
                s_wcls[p] = (uint8_t)c;
                atomicAdd(&s_wbin[c], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x < 64) {  // exclusive scan of the counters (wave 0; NBIN / 64 per lane)
            constexpr int PER = NBIN / 64;
            u32 v[PER], tot = 0;
#pragma unroll
            for (int q = 0; q < PER; ++q) { v[q] = s_wbin[threadIdx.x * PER + q]; tot += v[q]; }
            u32 incl = tot;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const u32 t = (u32)__shfl_up((int)incl, off);
                if ((int)threadIdx.x >= off) incl += t;
            }
            u32 ex = incl - tot;
#pragma unroll
            for (int q = 0; q < PER; ++q) { s_wbin[threadIdx.x * PER + q] = ex; ex += v[q]; }
        }
        __syncthreads();
        for (int k = 0; k < (int)wt; ++k) {
            const u32 p = (u32)k * 256u + threadIdx.x;
            if (p < wn) s_ord[atomicAdd(&s_wbin[s_wcls[p]], 1u)] = (uint16_t)p;
        }
        __syncthreads();
    }
    for (int wk = 0; wk < (int)wt; ++wk) {
        u64 rel;
        bool live;
        if constexpr (SORT) {
            const u32 p = (u32)wk * 256u + q64 + (u32)me;
            live = p < wn;
            if constexpr (PRESORT) rel = win + (live ? (u32)B.word[win + p] : 0u);
            else rel = win + (live ? s_ord[p] : 0u);
        } else {
            rel = win + threadIdx.x;
            live = rel < nf;
        }
        u64 w[S];
        u32 m[K];
        const u32* rec = fr + (REP ? lo + rel : wslot(B, lo + rel)) * (u64)FW;
        if (live) {
            load_state<S, K>(rec, w, m);
        } else {
#pragma unroll
            for (int i = 0; i < S; ++i) w[i] = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) m[q] = 0;
        }
        // REP: the record's rank; only this rank's own states count as generated
        // (every rank expands every state) and as deadlocks
        u32 powner = B.rank;
        bool mine = true;
        if constexpr (REP) {
            powner = live ? (rec[RR::REF + 1] >> 16) & 0xFFu : B.rank;
            mine = powner == B.rank;
        }
        ParentMix<S, K> pmx;
        Fp h0;
        if constexpr (PRE) {
            parent_mix<S, K>(w, m, pmx);
            h0 = pmx.h0;
        } else {
            h0 = state_fp<S, K>(w, m);
        }
        // SYMMETRY: the parent's signature bases (reused by every lane)
        u64 sbase[SYM ? S : 1];
        if constexpr (SYM) {
#pragma unroll
            for (int i = 0; i < S; ++i) sbase[i] = sig_base<S>(w[i], (u32)i);
        }
        Diamond dm;  // DIA: how this state was discovered (lane + footprint), once per state
        if constexpr (DIA) {
            const bool on = live && P.diamond;
            int act = 255;
            u64 foot = 0;
            if (on) {
                if constexpr (REP) {
                    act = (int)(rec[RR::ACT] & 0xFFu);
                    foot = (u64)rec[RR::FOOT] | ((u64)rec[RR::FOOT + 1] << 32);
                } else {
                    act = (int)B.act[lo + rel];
                    foot = B.foot[wslot(B, lo + rel)];
                }
            }
            diamond_of<S, K>(m, act, foot, P, dm);
        }
        u32 g = 0;
        // SORT: the lanes some state of this wave can enable (wave-uniform, scalar;
        // wm_hi: lanes 64-127, shapes of more than 64 lanes only)
        constexpr bool WIDE_MASK = Lanes<S, K>::N > 64;
        u64 wm = 0, wm_hi = 0;
        if constexpr (SORT) {
            const LaneMask lm = lane_superset_wave<S, K>(w, m, P.V, live);
            wm = lm.lo;
            if constexpr (WIDE_MASK) wm_hi = lm.hi;
        }
#ifdef RMC_WALK_STATS_BUILD
        walked += live ? (u32)(SORT ? __popcll(wm) + __popcll(wm_hi) : nl) : 0u;  // per thread (a VGPR)
#endif
        for (int lane0 = 0; SORT ? ((wm | wm_hi) != 0) : (lane0 < nl); lane0 += BATCH) {  // wave-uniform (pr: probes)
            u64 lp = 0;  // SORT: this batch's lanes, 7 bits each (127 = none), a scalar
            if constexpr (SORT) {
#pragma unroll
                for (int b = 0; b < BATCH; ++b) {
                    u64 ln;
                    if constexpr (WIDE_MASK) {
                        ln = wm ? (u64)__builtin_ctzll(wm) : wm_hi ? 64ull + (u64)__builtin_ctzll(wm_hi) : 127ull;
                        if (wm) wm &= wm - 1;
                        else wm_hi &= wm_hi - 1;
                    } else {
                        ln = wm ? (u64)__builtin_ctzll(wm) : 127ull;
                        wm &= wm - 1;
                    }
                    lp |= ln << (7 * b);
                }
            }
            u64 cur_p[PIPE ? BATCH : 1];  // PIPE: the probes issued during (a)
            // (a) deltas + fingerprints of BATCH lanes; keys parked in LDS (0 = no probe).
            // Rolled under SYMMETRY: one copy of the canonicalisation in flight.
            // (Rolling the plain kernel too, one copy of the lane code instead of
            // 8, measured no difference: instruction-cache misses are ~1e-5.)
#ifndef RMC_LANE_UNROLL
#define RMC_LANE_UNROLL BATCH
#endif
            constexpr int UNROLL = SYM ? 1 : RMC_LANE_UNROLL;
#pragma unroll UNROLL
            for (int b = 0; b < BATCH; ++b) {
                const int lane = SORT ? (int)((lp >> (7 * b)) & 127u) : lane0 + b;
                u64 key = 0, slot0 = 0;  // the probe's table value (0: none) and first slot
                u32 ks = 0;
                int tied = 0;  // SYMMETRY: signatures tie, deferred to k_ties
                if (lane < nl) {
                    Delta d;
                    if constexpr (SORT) lane_delta_desc<S, K>(w, m, P.ldesc[SORT ? lane : 0], P, d);  // scalar descriptor
                    else lane_delta<S, K>(w, m, lane, P, d);
                    const int en = d.en && live;
                    g += (u32)(en && mine);
                    Fp h{0, 0};
                    u64 hwn = 0;  // DIST: the mix of the changed server word (owner routing)
                    int in_model = 0;
                    if constexpr (SYM) {
                        // a stutter (successor = parent: no bag change, no word change) is never probed
                        const bool stutter = d.rm < 0 && !d.has_add && (d.srv < 0 || d.w_new == selw<S>(w, d.srv));
                        if (en && !stutter && delta_in_model<S, K>(m, d, P)) {
                            in_model = 1;
                            if constexpr (TIEDEFER) {  // tied signatures: k_ties canonicalises it after this launch
                                h = canon_delta<S, K, true>(w, m, sbase, d, PT.code, PT.np, &tied);
                                if (tied) in_model = 0;
                            } else {
                                h = canon_delta<S, K>(w, m, sbase, d, PT.code, PT.np);
                            }
                        }
                    } else if (en) {
                        int nmb = 0;
                        if constexpr (PRE)
                            in_model = delta_fp_pre<S, K>(w, m, pmx, d, P, &h, DIA ? &nmb : nullptr,
                                                          (REP || SENTC) ? &hwn : nullptr);
                        else in_model = delta_fp<S, K>(w, m, h0, d, P, &h, DIA ? &nmb : nullptr);
                        if constexpr (DIA)
                            if (in_model && h.k != h0.k &&
                                (SORT ? diamond_skip_desc<S, K>(m, lane, P.ldesc[SORT ? lane : 0], d, nmb, dm)
                                      : diamond_skip<S, K>(m, lane, d, nmb, dm, P)))
                                in_model = 0;
                    }
                    if (in_model && (SYM || h.k != h0.k)) {  // (a stutter has the parent's k)
                        if constexpr (VERIFY) h = fp_weaken(h, P.fp_mask);
                        ks = fp_norm(h.k, (u32)h.s, B.tmask);
                        key = fp_v(h.k, ks, B.tmask);
                        slot0 = h.k & B.tmask;
                        if constexpr (REP) {  // a replicated level: only the owner probes
                            if (owner_succ<S, K>(h.k, d, pmx, hwn, B, powner) != B.rank) key = 0;
                        } else if constexpr (SENTC) {
                            if constexpr (PRE)
                                s_own[b][threadIdx.x] = (uint8_t)owner_succ<S, K>(h.k, d, pmx, hwn, B, B.rank);
                            else  // no parent mixes: the successor's words 0 and 1 when it changes one
                                s_own[b][threadIdx.x] = (uint8_t)(
                                    B.world == 1 ? 0u
                                    : B.owner_mode == 0 ? owner_of(h.k, B.world)
                                    : owner_succ_w<S>(h.k, d, w, B));
                        }
                    }
                }
                s_key[b][threadIdx.x] = key;
                s_ks[b][threadIdx.x] = ks;
                if constexpr (PIPE != 0) cur_p[b] = key ? B.table[slot0] : 0ull;
                if constexpr (TIEDEFER) {  // one queue atomic per wave and lane, not per tied successor
                    const u64 bal = __ballot(tied);
                    if (bal) {
                        const int leader = __ffsll((long long)bal) - 1;
                        u64 q0 = 0;
                        if (me == leader) q0 = atomicAdd((unsigned long long*)&B.ctr->nties, (unsigned long long)__popcll(bal));
                        q0 = bcast64(q0, leader);
                        if (tied) {
                            const u64 q = q0 + (u64)__popcll(bal & lt_mask);
                            if (q < B.tie_cap) B.ties[q] = (lo + rel) | ((u64)lane << 56);
                            else atomicOr(&B.ctr->overflow, 16u);
                        }
                    }
                }
            }
            // (b) BATCH independent first-slot probes in flight at once
            u64 key[BATCH], cur[BATCH];
#pragma unroll
            for (int b = 0; b < BATCH; ++b) {
                key[b] = s_key[b][threadIdx.x];
                if constexpr (SENTC) {
                    const bool remote = key[b] && s_own[b][threadIdx.x] != B.rank;
                    // no sent-cache in verification mode (B.sent null): every remote successor is shipped
                    cur[b] = !key[b] ? 0ull
                           : remote ? (B.sent ? B.sent[(key[b] >> 8) & B.smask] : 0ull)
                                    : B.table[fp_slot(key[b], s_ks[b][threadIdx.x], B.tmask)];
                } else if constexpr (PIPE != 0) {
                    cur[b] = cur_p[PIPE ? b : 0];
                } else {
                    cur[b] = key[b] ? B.table[fp_slot(key[b], s_ks[b][threadIdx.x], B.tmask)] : 0ull;
                }
            }
#pragma unroll
            for (int b = 0; b < BATCH; ++b) pr += (u64)__popcll(__ballot(key[b] != 0));  // wave-uniform
            // (c) resolve: hit -> duplicate; empty -> CAS; mismatch -> slow path
            u32 newbits = 0, slowbits = 0;
            u32 hitbits = 0;  // verification: probes that found their key (slot parked in s_key)
#pragma unroll
            for (int b = 0; b < BATCH; ++b) {
                if (!key[b]) continue;
                if (cur[b] == key[b]) {
                    if constexpr (VERIFY) {
                        hitbits |= 1u << b;
                        s_key[b][threadIdx.x] = fp_slot(key[b], s_ks[b][threadIdx.x], B.tmask);  // the key's slot
                    }
                    continue;
                }
                if constexpr (SENTC) {
                    if (s_own[b][threadIdx.x] != B.rank) {  // not sent before (lossy cache): ship it
                        if (B.sent) B.sent[(key[b] >> 8) & B.smask] = key[b];
                        newbits |= 1u << b;
                        continue;
                    }
                }
                if (fp_empty(cur[b])) {  // 0, or another epoch's entry: CAS it away
                    const u64 sl0 = fp_slot(key[b], s_ks[b][threadIdx.x], B.tmask);
                    const u64 prev = atomicCAS((unsigned long long*)&B.table[sl0], (unsigned long long)cur[b],
                                               (unsigned long long)key[b]);
                    if (prev == cur[b]) newbits |= 1u << b;
                    else if (prev != key[b]) slowbits |= 1u << b;
                    else if constexpr (VERIFY) {
                        hitbits |= 1u << b;
                        s_key[b][threadIdx.x] = sl0;
                    }
                } else {
                    slowbits |= 1u << b;
                }
            }
            while (slowbits) {  // rare: linear probing past an occupied first slot
                const int b = __builtin_ctz(slowbits);
                slowbits &= slowbits - 1;
                const u64 kv = s_key[b][threadIdx.x], sl0 = fp_slot(kv, s_ks[b][threadIdx.x], B.tmask);
                if constexpr (VERIFY) {
                    u64 at = 0;
                    if (fp_insert_at(B.table, B.tmask, sl0, kv, &B.ctr->table_full, &at)) {
                        newbits |= 1u << b;
                    } else {
                        hitbits |= 1u << b;
                        s_key[b][threadIdx.x] = at;  // the slot that holds the key
                    }
                } else if (fp_insert(B.table, B.tmask, sl0, kv, &B.ctr->table_full)) {
                    newbits |= 1u << b;
                }
            }
            if constexpr (VERIFY) {
                // compare each hit with the stored owner of its slot (parked in s_key)
                u32 defbits = 0, hostbits = 0;
                for (int b = 0; b < BATCH; ++b) {  // rolled: one inlined copy of the check
                    if (!((hitbits >> b) & 1u)) continue;
                    const int r = verify_hit<S, K, SYM>(w, m, lane0 + b, s_key[b][threadIdx.x], P, PT, B);
                    vchk += (u64)(r <= 1);
                    vcol += (u64)(r == 1);
                    defbits |= (u32)(r == 2) << b;
                    hostbits |= (u32)(r == 4) << b;
                }
                // owners that left the device window (spill): checked on their host
                // copies after the launch (k_verify_host)
                for (int b = 0; b < BATCH; ++b) {
                    const bool hd = (hostbits >> b) & 1u;
                    const u64 bal = __ballot(hd);
                    if (!bal) continue;
                    const int leader = __ffsll((long long)bal) - 1;
                    u64 q0 = 0;
                    if (me == leader) q0 = atomicAdd((unsigned long long*)&B.ctr->hcount, (unsigned long long)__popcll(bal));
                    q0 = bcast64(q0, leader);
                    if (hd) {
                        const u64 q = q0 + (u64)__popcll(bal & lt_mask);
                        if (q < B.hcap) {
                            B.hbuf[2 * q] = lo + rel;
                            B.hbuf[2 * q + 1] = B.sidx[s_key[b][threadIdx.x]] | ((u64)(lane0 + b) << 56);
                        } else {
                            atomicOr(&B.ctr->overflow, 4u);
                        }
                    }
                }
                // defer hits on owners not yet published (one atomic per wave and probe batch)
                for (int b = 0; b < BATCH; ++b) {
                    const bool def = (defbits >> b) & 1u;
                    const u64 bal = __ballot(def);
                    if (!bal) continue;
                    const int leader = __ffsll((long long)bal) - 1;
                    u64 q0 = 0;
                    if (me == leader) q0 = atomicAdd((unsigned long long*)&B.ctr->vcount, (unsigned long long)__popcll(bal));
                    q0 = bcast64(q0, leader);
                    if (def) {
                        const u64 q = q0 + (u64)__popcll(bal & lt_mask);
                        if (q < B.vcap) {
                            B.vbuf[2 * q] = lo + rel;
                            B.vbuf[2 * q + 1] = s_key[b][threadIdx.x] | ((u64)(lane0 + b) << 56);
                        } else {
                            atomicOr(&B.ctr->overflow, 4u);
                        }
                    }
                }
            }
            // (d) list the winners (wave-aggregated, no global atomics)
            for (int b = 0; b < BATCH; ++b) {
                const int is_new = (newbits >> b) & 1u;
                const u64 bal = __ballot(is_new);
                if (bal) {
                    if (is_new) {
                        const u32 pos = n + (u32)__popcll(bal & lt_mask);
                        l_rel[pos] = (u32)rel;
                        l_lane[pos] = (uint8_t)(SORT ? (int)((lp >> (7 * b)) & 127u) : lane0 + b);
                        if constexpr (SENTC) {
                            l_dest[pos] = s_own[b][threadIdx.x];
                            l_key[pos] = key[b];
                            l_ks[pos] = s_ks[b][threadIdx.x];
                        }
                    }
                    n += (u32)__popcll(bal);
                    if (n > (u32)(LCAP - 64)) {
                        if constexpr (REP) flush_new<S, K, true>(P, B, lo, l_rel, l_lane, n);
                        else if constexpr (POOL) flush_pool<S, K>(P, B, lo, l_rel, l_lane, l_dest, n);
                        else if constexpr (MARK) flush_mark<S, K>(P, B, lo, l_rel, l_lane, l_dest, n);
                        else if constexpr (DIST) flush_dist<S, K>(P, B, lo, l_rel, l_lane, l_dest, l_key, l_ks, n);
                        else flush_new<S, K>(P, B, lo, l_rel, l_lane, n);
                        n = 0;
                    }
                }
            }
        }
        if (live && mine && g == 0) {  // deadlock: the state's index on its own rank
            const u64 ix = REP ? (((u64)rec[RR::REF] | ((u64)rec[RR::REF + 1] << 32)) & ((1ull << 48) - 1)) : lo + rel;
            atomicMin((unsigned long long*)&B.ctr->deadlock, (unsigned long long)ix);
        }
        gen += g;
    }
    }
    if (n) {
        if constexpr (REP) flush_new<S, K, true>(P, B, lo, l_rel, l_lane, n);
        else if constexpr (POOL) flush_pool<S, K>(P, B, lo, l_rel, l_lane, l_dest, n);
        else if constexpr (MARK) flush_mark<S, K>(P, B, lo, l_rel, l_lane, l_dest, n);
        else if constexpr (DIST) flush_dist<S, K>(P, B, lo, l_rel, l_lane, l_dest, l_key, l_ks, n);
        else flush_new<S, K>(P, B, lo, l_rel, l_lane, n);
    }
    // wave reductions of the generated and probe counts, one atomic each per wave
    u64 gs = (u64)gen;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        gs += (u64)(u32)__shfl_xor((int)(u32)gs, off) | ((u64)(u32)__shfl_xor((int)(u32)(gs >> 32), off) << 32);
    if (me == 0 && gs) atomicAdd((unsigned long long*)&B.ctr->generated, (unsigned long long)gs);
    if (me == 0 && pr) atomicAdd((unsigned long long*)&B.ctr->probes, (unsigned long long)pr);
    const u64 wk_sum = wave_sum64((u64)walked);
    if (me == 0 && wk_sum) atomicAdd((unsigned long long*)&B.ctr->walked, (unsigned long long)wk_sum);
    if constexpr (VERIFY) {
        vchk = wave_sum64(vchk);
        vcol = wave_sum64(vcol);
        if (me == 0 && vchk) atomicAdd((unsigned long long*)&B.ctr->vchecked, (unsigned long long)vchk);
        if (me == 0 && vcol) atomicAdd((unsigned long long*)&B.ctr->collisions, (unsigned long long)vcol);
    }
}

// Depth-bounded unconstrained models (Params.unbounded): a successor that takes
// an unbounded field past the packed capacity stops the search with
// RMC_E_CAPACITY naming the field.  A separate pass over the launch's states,
// run only for such models, so the expansion kernels carry no code for it
// (in their lane loop it cost 8 % of the S = 5 kernel's instructions).
template <int S, int K>
__global__ __launch_bounds__(256) void k_capacity_check(const Params P, const DevBufs B, u64 lo, u64 hi) {
    constexpr int NW = 2 * S + K;
    const int nl = P.off[10];
    u32 bad = 0;
    for (u64 t = lo + (u64)blockIdx.x * 256 + threadIdx.x; t < hi; t += (u64)gridDim.x * 256) {
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + wslot(B, t) * (u64)NW, w, m);
        for (int lane = 0; lane < nl; ++lane) {
            Delta d;
            lane_delta<S, K>(w, m, lane, P, d);
            if (d.en) bad |= (u32)capacity_exceeded<S, K>(m, d, P);  // 0 for in-model successors
        }
    }
    if (bad) atomicOr(&B.ctr->overflow, bad << 8);
}

// Every lane of every state (shapes with more than 64 lanes; verification).
template <int S, int K, bool SYM, int BATCH, bool DIST, bool VERIFY = false, bool PRE = false>
__global__ __launch_bounds__(256) void k_expand(const Params P, const PermTable PT, const DevBufs B, u64 lo, u64 hi) {
    expand_body<S, K, SYM, BATCH, DIST, VERIFY, PRE>(P, PT, B, lo, hi);
}

// The single-GPU expansion kernel: the lane-superset walk over windows of 16
// tiles presorted by class (PS), commuting-diamond skipping, WPE waves/SIMD, DYN
// dynamic per-wave work units; PI: probe loads issued during the lane code (K = 8
// shapes would spill 10-13 VGPRs).
template <int S, int K, int BATCH, int PI, bool PS = false, int WPE = 4, bool PRE = true, int DYN = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_expand_sort(
    const Params P, const PermTable PT, const DevBufs B, u64 lo, u64 hi) {
    if constexpr (Lanes<S, K>::N <= 128)
        expand_body<S, K, false, BATCH, false, false, PRE, true, true, false, 16, PI, false, PS, DYN>(P, PT, B, lo,
                                                                                                     hi);
}

// SYMMETRY expansion: each lane fingerprints its successor under the
// permutation that sorts the servers by signature, all S! only on ties
// (deferred to k_ties).  WS: the lane-superset walk over class-sorted windows
// of 16 tiles, 4 waves/SIMD (72.1-72.7 vs 75.0-75.3 ms for 8 tiles on the
// MCraftBench bounds); otherwise (more than 64 lanes) every lane, 5 waves/SIMD.
// (Round 4: windows presorted by k_window_order, 6 probes, 5 waves/SIMD measured
// 78.0-78.5 vs 78.6-78.9 ms on the MCraftBench bounds, profiles/r04/ab/sym_variant_r04n.txt:
// neutral, removed.)
// PS (round 6, the default): the windows presorted by k_window_order, so the
// block carries no LDS sort (35 instead of 48 KB: the 96-bit keys' s_ks array
// had cut the in-kernel sort's block to 3 per CU, i.e. 3 waves/SIMD); with 6
// probes in flight (BATCH) the block takes 28.7 KB and the kernel runs at 5 waves.
template <int S, int K, int BATCH, bool WS, bool PS = false, int DYN = 0,
          int WPE = (S == 3 && K == 4 ? (WS ? 4 : 5) : 1)>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void
k_expand_sym(const Params P, const PermTable PT, const DevBufs B, u64 lo, u64 hi) {
    if constexpr (WS && PS && Lanes<S, K>::N <= 128)
        expand_body<S, K, true, BATCH, false, false, false, true, false, false, 16, 0, false, true, DYN>(P, PT, B, lo,
                                                                                                       hi);
    else if constexpr (WS && Lanes<S, K>::N <= 128)
        expand_body<S, K, true, BATCH, false, false, false, true, false, false, 16>(P, PT, B, lo, hi);
    else
        expand_body<S, K, true, BATCH, false, false, false>(P, PT, B, lo, hi);
}



// The sharded expansion: send markers in the local set, diamond skipping and
// the lane-superset walk over class-sorted windows of 8 tiles (4 waves/SIMD;
// uncapped it takes 131 VGPRs: 3 waves); every lane for more than 64 lanes.
// REP: a replicated level (the whole level's records in B.rep).
// POOL: the pool flush (flush_pool) with the single-GPU kernel's shape (presorted
// windows of 16 tiles, early probe loads, the parent's mixes recomputed per lane).
template <int S, int K, int BATCH, bool REP, bool PS = false, int WPE = 4, bool POOL = false, int DYN = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_expand_dist(
    const Params P, const PermTable PT, const DevBufs B, u64 lo, u64 hi) {
    if constexpr (Lanes<S, K>::N <= 128 && POOL && !REP)
        expand_body<S, K, false, BATCH, true, false, false, true, true, true, 16, K <= 4 ? 1 : 0, false, true, DYN,
                    true>(P, PT, B, lo, hi);
    else if constexpr (POOL && !REP)  // more than 64 lanes: every lane, the pool flush
        expand_body<S, K, false, BATCH, true, false, false, false, false, true, 8, 0, false, false, 0, true>(P, PT, B,
                                                                                                           lo, hi);
    else if constexpr (Lanes<S, K>::N <= 128)
        expand_body<S, K, false, BATCH, true, false, true, true, true, true, 8, 0, REP>(P, PT, B, lo, hi);
    else if constexpr (!REP)
        expand_body<S, K, false, BATCH, true, false, false, false, false, true>(P, PT, B, lo, hi);
}

#ifndef RMC_SHAPE_S  // non-template kernels: in the common object only
// Sharded mode, phase 1, owner side: insert the keys other ranks sent;
// reply[t] = 1 if key t was new here (its sender then ships the state), and
// acc[p] counts the new keys of source p — the states p will send in phase 2,
// so the receive sizes need no second count exchange.  Keys arrive grouped by
// source, so a wave mostly adds to one counter (one atomic per source present).
__global__ __launch_bounds__(256) void k_owner_insert(const DevBufs B, const u32* keys, uint8_t* reply, u64 n,
                                                      const SrcOff so, unsigned long long* acc) {
    u64 pr = 0;
    const int me = (int)__lane_id();
    for (u64 t0 = (u64)blockIdx.x * 256ull; t0 < n; t0 += (u64)gridDim.x * 256ull) {
        const u64 t = t0 + threadIdx.x;
        u32 src = 0xFFFFFFFFu;
        if (t < n) {
            const u32* kr = keys + 3 * t;  // {k lo, k hi, s32}
            const int isnew = fp_insert_fp(B.table, B.tmask, Fp{(u64)kr[0] | ((u64)kr[1] << 32), kr[2]},
                                           &B.ctr->table_full);
            reply[t] = (uint8_t)isnew;
            if (isnew) {
                u32 p = 0;
                while (p + 1 < B.world && so.o[p + 1] <= t) ++p;
                src = p;
            }
        }
        pr += (u64)__popcll(__ballot(t < n));
        u64 pending = __ballot(src != 0xFFFFFFFFu);
        while (pending) {  // wave-uniform
            const int l = __ffsll((long long)pending) - 1;
            const u32 s = (u32)__builtin_amdgcn_readlane((int)src, l);
            const u64 bal = __ballot(src == s);
            if (me == l) atomicAdd(&acc[s], (unsigned long long)__popcll(bal));
            pending &= ~bal;
        }
    }
    if (me == 0 && pr) atomicAdd((unsigned long long*)&B.ctr->probes, (unsigned long long)pr);
}

// Presorted windows (k_expand_sort<PS>): the frontier [lo, lo + nf) cut into
// the windows the expansion kernel will take (256 * wt states, wt from the
// launch size and the expansion grid exactly as the kernel computes it), each
// counting-sorted by the states' 1-byte classes: word[win + i] = the i-th
// position of window win in class order.
// The lanes of the wave holding the same 8-bit class as this one (one ballot
// per class bit; inactive lanes never match).
__device__ __forceinline__ u64 match_class8(u32 c, bool act) {
    u64 peers = __ballot(act);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const u64 on = __ballot(act && ((c >> b) & 1u));
        peers &= ((c >> b) & 1u) ? on : ~on;
    }
    return peers;
}

// The class counters take one LDS atomic per class present in a wave's 64
// positions (match_class8), not one per position: a window's states fall in a
// few classes, and same-address LDS atomics serialise (0.91 bank conflicts per
// LDS access with per-position atomics, round 4's PMC profile).
// Round 6: every class byte of the thread's window positions is loaded up front
// (16 independent loads, one memory latency per window instead of one per
// 256-position round), each position's peers (match_class8) are found once and
// kept for the scatter pass, and the grid is one round of resident blocks of
// this kernel rather than of the expansion kernel.
__global__ __launch_bounds__(256) void k_window_order(const uint8_t* cls, u64 wmask, u64 lo, u64 nf, u64 wt,
                                                      uint16_t* word, unsigned long long* wnext) {
    __shared__ u32 bins[256];
    const u32 tid = threadIdx.x;
    const u64 lt = (1ull << __lane_id()) - 1ull;
    if (blockIdx.x == 0 && tid == 0) *wnext = 0;  // the next expansion launch's dynamic work counter
    for (u64 win = (u64)blockIdx.x * 256ull * wt; win < nf; win += (u64)gridDim.x * 256ull * wt) {
        const u32 wn = (u32)((nf - win) < 256ull * wt ? (nf - win) : 256ull * wt);
        u32 cv[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const u32 p = (u32)k * 256u + tid;
            cv[k] = p < wn ? (u32)cls[(lo + win + p) & wmask] : 0u;
        }
        __syncthreads();
        bins[tid] = 0;
        __syncthreads();
        // pass 1: one counter atomic per class present in a wave's 64 positions; each
        // position keeps class | rank among its peers << 8 | their leader << 14 | their number << 20
#pragma unroll
        for (int k = 0; k < 16; ++k) {  // block-uniform rounds
            if ((u32)k * 256u >= wn) break;
            const bool act = (u32)k * 256u + tid < wn;
            const u32 c = cv[k];
            const u64 peers = match_class8(c, act);
            const u32 rank = (u32)__popcll(peers & lt), cnt = (u32)__popcll(peers);
            if (act && rank == 0) atomicAdd(&bins[c], cnt);
            const u32 leader = peers ? (u32)(__ffsll((long long)peers) - 1) : 0u;
            cv[k] = c | (rank << 8) | (leader << 14) | (cnt << 20);
        }
        __syncthreads();
        if (tid < 64) {  // exclusive scan of the 256 counters: 4 per lane, then across the wave
            u32 v[4], tot = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) { v[q] = bins[tid * 4 + q]; tot += v[q]; }
            u32 incl = tot;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const u32 t = (u32)__shfl_up((int)incl, off);
                if ((int)tid >= off) incl += t;
            }
            u32 ex = incl - tot;
#pragma unroll
            for (int q = 0; q < 4; ++q) { bins[tid * 4 + q] = ex; ex += v[q]; }
        }
        __syncthreads();
        // pass 2: the leader of each class group reserves its group's positions
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if ((u32)k * 256u >= wn) break;
            const u32 p = (u32)k * 256u + tid;
            const bool act = p < wn;
            const u32 v = cv[k], c = v & 0xFFu, rank = (v >> 8) & 63u, leader = (v >> 14) & 63u, cnt = v >> 20;
            u32 base = 0;
            if (act && rank == 0) base = atomicAdd(&bins[c], cnt);
            base = (u32)__shfl((int)base, (int)leader);
            if (act) word[win + base + rank] = (uint16_t)p;
        }
    }
}

static u64 resident_grid(const void* k);  // (host launchers, below)
hipError_t launch_window_order(const DevBufs& B, u64 lo, u64 hi, u64 grid, u64 wt_max, hipStream_t st) {
    const u64 nf = hi - lo;
    if (nf == 0) return hipSuccess;
    if (wt_max > 16 || nf > (1ull << kMaxLaunchLog2)) return hipErrorInvalidValue;
    // the expansion kernel's window size for this launch (expand_body: per_block)
    const u64 per_block = (nf + grid * 256ull - 1) / (grid * 256ull);
    const u64 wt = per_block < wt_max ? (per_block ? per_block : 1ull) : wt_max;
    const u64 nwin = (nf + 256ull * wt - 1) / (256ull * wt);
    // its own grid: one round of its resident blocks (RMC_WORDER_GRID=0: the expansion's, round 5)
    static const u64 og = [] {
        const char* e = getenv("RMC_WORDER_GRID");
        return e ? (u64)atoll(e) : (u64)1;
    }();
    const u64 g2 = og == 0 ? grid : og == 1 ? resident_grid(reinterpret_cast<const void*>(&k_window_order)) : og;
    hipLaunchKernelGGL(k_window_order, dim3((unsigned)(nwin < g2 ? nwin : g2)), dim3(256), 0, st, B.cls, B.wmask, lo, nf,
                       wt, B.word, (unsigned long long*)&B.ctr->wnext);
    return hipGetLastError();
}

// Sharded mode: the count row of one exchange round (launch_pack_counts): a
// block of kRowWords u64 per peer — keys for it, flags, this rank's counters —
// then novf.
__global__ void k_pack_counts(const DevBufs B, u64 host_more, u64 ovf_done, u64* out, u64* mirror) {
    const u32 p = threadIdx.x;
    const u64 novf = B.ctr->novf;
    bool sends = false;
    for (u32 q = 0; q < B.world; ++q) sends |= q != B.rank && B.ocount[q] != 0;
    // bit 0: more to send this level; bit 1: the parking buffer overflowed (every
    // rank reads every row and fails alike); bit 2: keys to some peer this round
    const u64 flags = host_more | (novf > ovf_done ? 1ull : 0ull) | (novf > B.ovf_cap ? 2ull : 0ull) |
                      (sends ? 4ull : 0ull);
    if (p < B.world) {
        u64* r = out + (u64)p * kRowWords;
        const u64 c = B.ocount[p];
        r[0] = p == B.rank ? 0ull : (c < B.kcap ? c : B.kcap);
        r[1] = flags;
        const u64* k = reinterpret_cast<const u64*>(B.ctr);
        for (int i = 0; i < kRowWords - 2; ++i) r[2 + i] = k[i];
        if (mirror)
            for (int i = 0; i < kRowWords; ++i) mirror[(u64)p * kRowWords + i] = r[i];
    }
    if (p == 0) out[(u64)kRowWords * B.world] = novf;
    if (mirror) __threadfence_system();  // the row is in pinned host memory: visible before the event
}

// Sharded mode: parked keys ovf[a, a + n) back into the outbox (n <= kcap, so
// no destination can overflow; ocount was zeroed for this round).
__global__ __launch_bounds__(256) void k_drain(const DevBufs B, u64 a, u64 n) {
    for (u64 t = (u64)blockIdx.x * 256ull + threadIdx.x; t < n; t += (u64)gridDim.x * 256ull) {
        const u64* r = B.ovf + 3 * (a + t);
        const u64 k = r[0], sf = r[1], tk = r[2];
        const u32 dest = (u32)((tk >> 48) & 0xFFu);
        const u64 slot = atomicAdd(&B.ocount[dest], 1ull);
        if (slot >= B.kcap) {  // cannot happen for n <= kcap; never write past the outbox
            atomicOr(&B.ctr->overflow, 2u);
            continue;
        }
        put_key(B, dest, slot, k, (u32)sf, (tk & ((1ull << 48) - 1)) | (tk & (0xFFull << 56)));
    }
}

#endif  // !RMC_SHAPE_S

// Sharded mode, after a pool-flush expansion (k_expand_dist<POOL>): every pool
// record [0, npool) gets its key (the state's fingerprint: order-free, so equal
// to the incremental probe key) and owner and goes to that owner's outbox as
// POOL_TICK | index, one reservation atomic per destination present in a wave;
// what does not fit is parked as a parent ticket (the pool is reused by the
// round after next, the parent store is not).
template <int S, int K>
__global__ __launch_bounds__(256) void k_route(const Params P, const DevBufs B) {
    constexpr int NW = 2 * S + K, RW = NW + 4;
    const int me = (int)__lane_id();
    const u64 lt = (1ull << me) - 1ull;
    const u64 np = *B.npool < B.pool_cap ? *B.npool : B.pool_cap;
    for (u64 t0 = (u64)blockIdx.x * 256ull; t0 < np; t0 += (u64)gridDim.x * 256ull) {  // wave-uniform
        const u64 t = t0 + threadIdx.x;
        const bool live = t < np;
        Fp key{0, 0};
        u64 ref = 0;
        u32 dest = 0xFFFFFFFFu;
        if (live) {
            const u32* r = B.pool + t * (u64)RW;
            u64 w[S];
            u32 m[K];
            load_state<S, K>(r, w, m);
            key = fp_of_materialised<S, K>(w, m, P);
            dest = owner_state<S>(key.k, w, B);
            ref = (u64)r[NW] | ((u64)r[NW + 1] << 32);
        }
        u64 slot = ~0ull;
        u64 pending = __ballot(live);
        while (pending) {  // wave-uniform: one atomic per destination present
            const int l = __ffsll((long long)pending) - 1;
            const u32 dd = (u32)__builtin_amdgcn_readlane((int)dest, l);
            const u64 bal = __ballot(dest == dd);
            u64 base = 0;
            if (me == l) base = atomicAdd(&B.ocount[dd], (unsigned long long)__popcll(bal));
            base = bcast64(base, l);
            if (dest == dd) slot = base + (u64)__popcll(bal & lt);
            pending &= ~bal;
        }
        if (!live) continue;
        if (slot < B.kcap) {
            put_key(B, dest, slot, key.k, (u32)key.s, POOL_TICK | t);
            continue;
        }
        // the owner's outbox is full: park it with its parent ticket (a later round sends it)
        park_key(B, key.k, (u32)key.s,
                 (ref & ((1ull << 40) - 1)) | ((u64)dest << 48) | (((ref >> 40) & 0xFFull) << 56));
    }
}
// Before k_route: the tickets the expansion itself parked (pool full) are
// OVF_UNKEYED until keyed here (k_route's own parked records carry theirs).
template <int S, int K>
__global__ __launch_bounds__(256) void k_route_fix(const Params P, const DevBufs B) {
    constexpr int NW = 2 * S + K;
    const u64 nov = B.ctr->novf < B.ovf_cap ? B.ctr->novf : B.ovf_cap;
    for (u64 q = (u64)blockIdx.x * 256ull + threadIdx.x; q < nov; q += (u64)gridDim.x * 256ull) {
        if (!(B.ovf[3 * q + 1] & OVF_UNKEYED)) continue;
        const u64 tk = B.ovf[3 * q + 2];
        const u64 pidx = tk & ((1ull << 48) - 1);
        const int lane = (int)(tk >> 56);
        u64 w[S], wo[S];
        u32 m[K], mo[K];
        load_state<S, K>(B.store + pidx * (u64)NW, w, m);
        Delta d;
        lane_delta<S, K>(w, m, lane, P, d);
        materialise<S, K>(w, m, d, wo, mo);
        const Fp key = fp_of_materialised<S, K>(wo, mo, P);
        B.ovf[3 * q] = key.k;
        B.ovf[3 * q + 2] = pidx | ((u64)owner_state<S>(key.k, wo, B) << 48) | ((u64)lane << 56);
        B.ovf[3 * q + 1] = (u32)key.s;
    }
}

// Sharded mode, phase 2, sender side: for every key an owner accepted
// (reply[d * kcap + i] = 1), re-derive the successor from its ticket and put
// the record {state, global parent ref | lane << 40} into owner d's state
// outbox.  Grid over (destination, key index).
// Full-state verification (B.sidx set): every key is shipped, the ones the
// owner had seen flagged REF_SEEN (parent-ref word), so the owner compares them with its state.
template <int S, int K>
__global__ __launch_bounds__(256) void k_materialize_remote(const Params P, const DevBufs B, const uint8_t* reply,
                                                            u64 per_dest, u64 i0) {
    constexpr int NW = 2 * S + K, RW = NW + 4;  // state, parent ref, footprint
    const u64 total = per_dest * B.world;  // window [i0, i0 + per_dest) of every destination's keys
    for (u64 t = (u64)blockIdx.x * 256ull + threadIdx.x; t < total; t += (u64)gridDim.x * 256ull) {
        const u32 d = (u32)(t / per_dest);
        const u64 i = i0 + (t - (u64)d * per_dest);
        const u64 sent = B.ocount[d] < B.kcap ? B.ocount[d] : B.kcap;  // beyond kcap: parked, not sent
        if (d == B.rank || i >= sent) continue;
        const bool seen = !reply[(u64)d * B.kcap + i];
        if (seen && !B.sidx) continue;
        const u64 tick = B.tick_out[(u64)d * B.kcap + i];
        const u64 pidx = tick & ((1ull << 48) - 1);
        const int lane = (int)(tick >> 56);
        const u64 slot = atomicAdd((unsigned long long*)&B.scount[d], 1ull);
        if (slot >= B.scap) {
            atomicOr(&B.ctr->overflow, 2u);
            continue;
        }
        if (tick & POOL_TICK) {  // a pool record is already the phase-2 record (never REF_SEEN: no verification)
            const uint2* src = reinterpret_cast<const uint2*>(B.pool + pidx * (u64)RW);
            uint2* dst = reinterpret_cast<uint2*>(B.st_out + ((u64)d * B.scap + slot) * (u64)RW);
#pragma unroll
            for (int q = 0; q < RW / 2; ++q) dst[q] = src[q];
            continue;
        }
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + pidx * (u64)NW, w, m);
        Delta dl;
        lane_delta<S, K>(w, m, lane, P, dl);
        u64 wo[S];
        u32 mo[K];
        materialise<S, K>(w, m, dl, wo, mo);
        u32* r = B.st_out + ((u64)d * B.scap + slot) * (u64)RW;
        store_state<S, K>(r, wo, mo);
        const u64 ref = B.ref_tag | ((u64)lane << 40) | pidx | (seen ? REF_SEEN : 0ull);
        r[NW] = (u32)ref;
        r[NW + 1] = (u32)(ref >> 32);
        const u64 ft = make_foot<S, K>(m, lane, dl, P);
        r[NW + 2] = (u32)ft;
        r[NW + 3] = (u32)(ft >> 32);
    }
}

// Sharded mode, phase 2, owner side: store the n accepted states received (their
// keys are already in this rank's set since phase 1): one allocation atomic per
// wave, parent ref and lane from the record, fused invariants.
template <int S, int K>
__global__ __launch_bounds__(256) void k_store_remote(const Params P, const DevBufs B, const u32* inbox, u64 n) {
    constexpr int NW = 2 * S + K, RW = NW + 4;  // state, parent ref, footprint
    const int me = (int)__lane_id();
    const u64 lt = (1ull << me) - 1ull;
    for (u64 t0 = (u64)blockIdx.x * 256ull; t0 < n; t0 += (u64)gridDim.x * 256ull) {
        const u64 t = t0 + threadIdx.x;
        // verification mode also receives the states the owner had seen (compared by k_compare_remote)
        const bool live = t < n && !(inbox[t * (u64)RW + NW + 1] & (u32)(REF_SEEN >> 32));
        const u64 bal = __ballot(live);
        if (!bal) continue;
        const int leader = __ffsll((long long)bal) - 1;
        u64 base = 0;
        if (me == leader) base = atomicAdd((unsigned long long*)&B.ctr->count, (unsigned long long)__popcll(bal));
        base = bcast64(base, leader);
        if (!live) continue;
        const u64 ni = base + (u64)__popcll(bal & lt);
        if (ni >= B.cap) {
            atomicOr(&B.ctr->overflow, 1u);
            continue;
        }
        const u32* r = inbox + t * (u64)RW;
        u64 w[S];
        u32 m[K];
        load_state<S, K>(r, w, m);
        const u64 ref = (u64)r[NW] | ((u64)r[NW + 1] << 32);
        store_new<S, K>(P, B, ni, w, m, ref & ~((0xFFull << 40) | REF_SEEN), (int)((ref >> 40) & 0xFFu),
                        (u64)r[NW + 2] | ((u64)r[NW + 3] << 32));
    }
}

// Sharded full-state verification, owner side: every received record the
// owner had already seen (REF_SEEN) is compared with the stored state that
// owns its fingerprint's slot (published by k_publish before this runs); a
// difference is a fingerprint collision.
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_compare_remote(const Params P, const PermTable PT, const DevBufs B,
                                                        const u32* inbox, u64 n) {
    constexpr int NW = 2 * S + K, RW = NW + 4;
    u64 vchk = 0, vcol = 0;
    for (u64 t = (u64)blockIdx.x * 256ull + threadIdx.x; t < n; t += (u64)gridDim.x * 256ull) {
        const u32* r = inbox + t * (u64)RW;
        if (!(r[NW + 1] & (u32)(REF_SEEN >> 32))) continue;
        PackedState<S, K> o;
        load_state<S, K>(r, o.w, o.m);
        const TKey key = verify_key<S, K, SYM>(o.w, o.m, P, PT, B.tmask);
        u64 s = key.s0, k = 0;
        while (B.table[s] != key.v && k <= B.tmask) { s = (s + 1) & B.tmask; ++k; }
        const u64 ix = k > B.tmask ? ~0ull : B.sidx[s];
        if (ix == ~0ull) {
            atomicOr(&B.ctr->overflow, 8u);  // a seen key without a published owner
            continue;
        }
        ++vchk;
        bool same;
        if constexpr (SYM) same = same_orbit<S, K>(o, B.store + ix * (u64)NW, PT);
        else same = same_state<S, K>(o.w, o.m, B.store + ix * (u64)NW);
        vcol += same ? 0u : 1u;
    }
    vchk = wave_sum64(vchk);
    vcol = wave_sum64(vcol);
    if (__lane_id() == 0 && vchk) atomicAdd((unsigned long long*)&B.ctr->vchecked, (unsigned long long)vchk);
    if (__lane_id() == 0 && vcol) atomicAdd((unsigned long long*)&B.ctr->collisions, (unsigned long long)vcol);
}

// SYMMETRY, single GPU: the successors k_expand_sym deferred because their
// server signatures tie.  Each is re-derived from its parent, canonicalised
// over every order of the tied servers, inserted, and committed if new.
template <int S, int K>
__global__ __launch_bounds__(256) void k_ties(const Params P, const PermTable PT, const DevBufs B) {
    constexpr int NW = 2 * S + K;
    const u64 n = B.ctr->nties < B.tie_cap ? B.ctr->nties : B.tie_cap;
    u64 pr = 0;
    for (u64 t0 = (u64)blockIdx.x * 256ull; t0 < n; t0 += (u64)gridDim.x * 256ull) {  // wave-uniform
        const u64 t = t0 + threadIdx.x;
        const bool live = t < n;
        u64 w[S];
        u32 m[K];
        u64 pidx = 0;
        int lane = 0;
        Delta d;
        int is_new = 0;
        if (live) {
            const u64 rec = B.ties[t];
            pidx = rec & ((1ull << 56) - 1);
            lane = (int)(rec >> 56);
            load_state<S, K>(B.store + wslot(B, pidx) * (u64)NW, w, m);
            lane_delta<S, K>(w, m, lane, P, d);
            u64 base[S];
#pragma unroll
            for (int i = 0; i < S; ++i) base[i] = sig_base<S>(w[i], (u32)i);
            is_new = fp_insert_fp(B.table, B.tmask, canon_delta<S, K>(w, m, base, d, PT.code, PT.np),
                                  &B.ctr->table_full);
        } else {
#pragma unroll
            for (int i = 0; i < S; ++i) w[i] = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) m[q] = 0;
            d.srv = -1; d.rm = -1; d.has_add = 0; d.add = 0; d.en = 0; d.w_new = 0;
        }
        pr += (u64)__popcll(__ballot(live));
        commit_new<S, K>(is_new, w, m, d, P, B, B.ref_tag | pidx, lane);
    }
    if (__lane_id() == 0 && pr) atomicAdd((unsigned long long*)&B.ctr->probes, (unsigned long long)pr);
}

// Probe-rate microbenchmark (the roofline ceiling for k_expand): every thread
// issues `iters` rounds of BATCH independent random 8-byte accesses into a
// table of `mask + 1` slots — plain loads (mode 0) or CAS (mode 1) — the
// access pattern of the fingerprint set, with no successor computation.
template <int BATCH>
__global__ __launch_bounds__(256) void k_probe_bench(u64* table, u64 mask, u32 iters, int mode, u64* sink) {
    const u64 t = (u64)blockIdx.x * 256ull + threadIdx.x;
    u64 acc = 0;
    for (u32 it = 0; it < iters; ++it) {
        u64 v[BATCH];
#pragma unroll
        for (int b = 0; b < BATCH; ++b) {
            const u64 key = mix64(t * 0x9E3779B97F4A7C15ull + (u64)it * BATCH + b) | 1ull;
            if (mode == 0) v[b] = table[key & mask];
            else v[b] = atomicCAS((unsigned long long*)&table[key & mask], 0ull, (unsigned long long)key);
        }
#pragma unroll
        for (int b = 0; b < BATCH; ++b) acc ^= v[b];
    }
    if (acc == 0x5A5A5A5A5A5A5A5Aull) sink[0] = acc;  // keeps the loads live
}

#ifndef RMC_SHAPE_S
hipError_t launch_owner_insert(const DevBufs& B, const u64* keys, uint8_t* reply, u64 n, const SrcOff& so,
                               unsigned long long* acc, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const u64 blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_owner_insert, dim3((unsigned)(blocks < 2048 ? blocks : 2048)), dim3(256), 0, st, B,
                       reinterpret_cast<const u32*>(keys), reply, n, so, acc);
    return hipGetLastError();
}

hipError_t launch_pack_counts(const DevBufs& B, u64 host_more, u64 ovf_done, u64* out, hipStream_t st, u64* mirror) {
    if (B.world > (u32)kMaxWorld) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_pack_counts, dim3(1), dim3(64), 0, st, B, host_more, ovf_done, out, mirror);
    return hipGetLastError();
}

hipError_t launch_drain(const DevBufs& B, u64 a, u64 n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const u64 blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_drain, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, st, B, a, n);
    return hipGetLastError();
}

// Clears the fingerprint set (or writes the verification slot map's 0xFF) at
// the start of a run: 16-B nontemporal stores, each thread four per round,
// consecutive across the block, the rounds strided over a fixed grid.  The
// run-start clear of the 69-GB XL set is 1.5 % of its BFS (verdict r05).
typedef u32 v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void __launch_bounds__(256) k_fill(v4u* p, u64 n16, u32 pat) {
    const v4u x = {pat, pat, pat, pat};
    const u64 stride = (u64)gridDim.x * 1024ull;
    for (u64 i = (u64)blockIdx.x * 1024ull + threadIdx.x; i < n16; i += stride) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u64 q = i + (u64)j * 256ull;
            if (q < n16) {
                if constexpr (NT) __builtin_nontemporal_store(x, p + q);
                else p[q] = x;
            }
        }
    }
}

hipError_t launch_fill(void* p, u64 bytes, uint8_t byte, hipStream_t st) {
    static const int mode = [] {  // RMC_FILL=0: hipMemsetAsync (the A/B baseline), 1 nontemporal, 2 plain stores
        const char* e = getenv("RMC_FILL");
        return e ? atoi(e) : 1;
    }();
    const u64 n16 = mode ? bytes / 16 : 0;
    if (n16) {
        const u64 blocks = (n16 + 1023) / 1024;
        const u32 pat = 0x01010101u * byte;
        const dim3 g((unsigned)(blocks < 4096 ? blocks : 4096));
        if (mode == 1) hipLaunchKernelGGL(k_fill<true>, g, dim3(256), 0, st, static_cast<v4u*>(p), n16, pat);
        else hipLaunchKernelGGL(k_fill<false>, g, dim3(256), 0, st, static_cast<v4u*>(p), n16, pat);
        if (hipError_t e = hipGetLastError()) return e;
    }
    if (bytes > n16 * 16) return hipMemsetAsync(static_cast<char*>(p) + n16 * 16, byte, bytes - n16 * 16, st);
    return hipSuccess;
}

hipError_t launch_probe_bench(u64* table, u64 mask, u64 threads, u32 iters, int mode, u64* sink, hipStream_t st) {
    hipLaunchKernelGGL((k_probe_bench<8>), dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, table, mask,
                       iters, mode, sink);
    return hipGetLastError();
}

#endif  // !RMC_SHAPE_S

// Insert n staged initial states (packed) into the set and the store.
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_seed(const Params P, const PermTable PT, const DevBufs B, const u32* staged,
                                              u64 n) {
    constexpr int NW = 2 * S + K;
    const u64 t = (u64)blockIdx.x * 256ull + threadIdx.x;
    const bool live = t < n;
    u64 w[S];
    u32 m[K];
    if (live) {
        load_state<S, K>(staged + t * (u64)NW, w, m);
    } else {
#pragma unroll
        for (int i = 0; i < S; ++i) w[i] = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) m[q] = 0;
    }
    int is_new = 0;
    if (live) {
        // fp_weaken: a no-op unless a verification test weakens the fingerprint
        const Fp key = fp_weaken(SYM ? canon_state<S, K>(w, m, PT.code, PT.np) : state_fp<S, K>(w, m), P.fp_mask);
        // sharded mode: only the owner of an initial state stores it
        if (owner_state<S>(key.k, w, B) == B.rank) is_new = fp_insert_fp(B.table, B.tmask, key, &B.ctr->table_full);
    }
    Delta d;  // identity delta: the state itself
    d.srv = -1; d.rm = -1; d.has_add = 0; d.add = 0; d.en = 1; d.w_new = 0;
    commit_new<S, K>(is_new, w, m, d, P, B, ~0ull, 255);
}

// Recovery (rmc_recover): re-insert the keys of the stored states [lo, hi)
// into an empty fingerprint set — the set is rebuilt, not checkpointed.
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_rehash(const Params P, const PermTable PT, const DevBufs B, u64 lo, u64 hi) {
    constexpr int NW = 2 * S + K;
    for (u64 i = lo + (u64)blockIdx.x * 256ull + threadIdx.x; i < hi; i += (u64)gridDim.x * 256ull) {
        u64 w[S];
        u32 m[K];
        load_state<S, K>(B.store + wslot(B, i) * (u64)NW, w, m);
        const Fp key = fp_weaken(SYM ? canon_state<S, K>(w, m, PT.code, PT.np) : state_fp<S, K>(w, m), P.fp_mask);
        if (!fp_insert_fp(B.table, B.tmask, key, &B.ctr->table_full)) atomicOr(&B.ctr->overflow, 8u);  // duplicate
    }
}

// Replicated level (sharded mode): this rank's frontier states [lo, hi) as
// records for the level's all-gather (RepRec: state, global ref, footprint,
// lane | class << 8).
template <int S, int K>
__global__ __launch_bounds__(256) void k_pack_rep(const DevBufs B, u64 lo, u64 hi, u32* out) {
    constexpr int NW = 2 * S + K;
    typedef RepRec<S, K> RR;
    for (u64 i = lo + (u64)blockIdx.x * 256ull + threadIdx.x; i < hi; i += (u64)gridDim.x * 256ull) {
        u32* r = out + (i - lo) * (u64)RR::RR;
        const uint2* src = reinterpret_cast<const uint2*>(B.store + i * (u64)NW);
        uint2* dst = reinterpret_cast<uint2*>(r);
#pragma unroll
        for (int q = 0; q < NW / 2; ++q) dst[q] = src[q];
        const u64 ref = B.ref_tag | i;
        const u64 f = B.foot[i];
        r[RR::REF] = (u32)ref;
        r[RR::REF + 1] = (u32)(ref >> 32);
        r[RR::FOOT] = (u32)f;
        r[RR::FOOT + 1] = (u32)(f >> 32);
        r[RR::ACT] = (u32)B.act[i] | ((u32)B.cls[i] << 8);
        r[RR::ACT + 1] = 0;
    }
}

// Every enabled lane of n given states, written out without dedup.
template <int S, int K, bool SYM>
__global__ __launch_bounds__(256) void k_list(const Params P, const PermTable PT, const u32* in, u64 n, u32* out,
                                              u64 cap, unsigned long long* count) {
    constexpr int NW = 2 * S + K;
    constexpr int RW = 6 + NW;  // record: parent(2) lane(1) flags(1) fp(2) + state
    const u64 t = (u64)blockIdx.x * 256ull + threadIdx.x;
    if (t >= n) return;
    u64 w[S];
    u32 m[K];
    load_state<S, K>(in + t * (u64)NW, w, m);
    const Fp h0 = state_fp<S, K>(w, m);
    u64 sbase[S];
#pragma unroll
    for (int i = 0; i < S; ++i) sbase[i] = sig_base<S>(w[i], (u32)i);
    const int nl = P.off[10];  // == Lanes<S,K>::N; runtime on purpose (see lane_delta)
#pragma unroll 1
    for (int lane = 0; lane < nl; ++lane) {
        Delta d;
        lane_delta<S, K>(w, m, lane, P, d);
        if (!d.en) continue;
        Fp h{0, 0};
        const int in_model = delta_fp<S, K>(w, m, h0, d, P, &h);
        if (in_model) {
            if constexpr (SYM) h = canon_delta<S, K>(w, m, sbase, d, PT.code, PT.np);
        }
        const u64 o = atomicAdd(count, 1ull);
        if (o >= cap) continue;
        u32* r = out + o * (u64)RW;
        r[0] = (u32)t; r[1] = (u32)(t >> 32); r[2] = (u32)lane; r[3] = (u32)in_model;
        r[4] = (u32)h.k; r[5] = (u32)(h.k >> 32);
        u64 wo[S];
        u32 mo[K];
        if (in_model) {
            materialise<S, K>(w, m, d, wo, mo);
        } else {
#pragma unroll
            for (int i = 0; i < S; ++i) wo[i] = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) mo[q] = 0;
        }
#pragma unroll
        for (int i = 0; i < S; ++i) { r[6 + 2 * i] = (u32)wo[i]; r[7 + 2 * i] = (u32)(wo[i] >> 32); }
#pragma unroll
        for (int q = 0; q < K; ++q) r[6 + 2 * S + q] = mo[q];
    }
}

// ---- simulation (TLC -simulate; Smokeraft.cfg) -------------
// One thread per behaviour: a random initial state from `inits`, then up to
// depth-1 steps, each choosing uniformly (one reservoir pass over the lanes)
// among the enabled successors — mode 0: those within the packed capacity
// (term <= 15, Len(log) <= 3, <= K messages, count <= 3; P carries these
// bounds), mode 1: all of them, a chosen successor beyond the capacity ending
// the behaviour as "truncated".  No candidate ends it as "deadlocked"
// (Smokeraft.cfg:48 turns deadlock checking off).  Invariants are checked on
// every state.
// rec_beh >= 0: that behaviour also writes its states to rec (replay).
__device__ __forceinline__ u64 sim_rand(u64& x) {  // splitmix64 stream
    x += 0x9E3779B97F4A7C15ull;
    return mix64(x);
}

template <int S, int K>
__global__ __launch_bounds__(256) void k_simulate(const Params P, const u32* inits, u64 n_init, u64 n_beh, int depth,
                                                  u64 seed, int mode, SimCounters* out, i64 rec_beh, u32* rec) {
    constexpr int NW = 2 * S + K;
    u64 steps = 0, trunc = 0, dead = 0;
    for (u64 t = (u64)blockIdx.x * 256ull + threadIdx.x; t < n_beh; t += (u64)gridDim.x * 256ull) {
        if (rec_beh >= 0 && (i64)t != rec_beh) continue;  // replay of one behaviour
        u64 rs = mix64(seed ^ (t * 0xD1B54A32D192ED03ull));
        u64 w[S];
        u32 m[K];
        load_state<S, K>(inits + (sim_rand(rs) % n_init) * (u64)NW, w, m);
        const bool record = (i64)t == rec_beh;
        if (record) store_state<S, K>(rec, w, m);
        int v = check_invariants<S, K>(w, m, P);
        if (v) atomicMin((unsigned long long*)&out->viol, (unsigned long long)((1ull << 44) | ((u64)(v - 1) << 40) | t));
        for (int dd = 2; dd <= depth && !v; ++dd) {
            u32 cnt = 0;
            int pick = -1;
            for (int lane = 0; lane < P.off[10]; ++lane) {
                Delta d;
                lane_delta<S, K>(w, m, lane, P, d);
                if (!d.en) continue;
                Fp hh;
                if (mode == 0 && !delta_fp<S, K>(w, m, Fp{0, 0}, d, P, &hh)) continue;  // beyond the capacity
                ++cnt;
                if (sim_rand(rs) % cnt == 0) pick = lane;  // reservoir: uniform over enabled lanes
            }
            if (cnt == 0) {
                ++dead;
                break;
            }
            Delta d;
            lane_delta<S, K>(w, m, pick, P, d);
            Fp hh;
            if (!delta_fp<S, K>(w, m, Fp{0, 0}, d, P, &hh)) {
                ++trunc;
                break;
            }
            u64 wo[S];
            u32 mo[K];
            materialise<S, K>(w, m, d, wo, mo);
#pragma unroll
            for (int i = 0; i < S; ++i) w[i] = wo[i];
#pragma unroll
            for (int q = 0; q < K; ++q) m[q] = mo[q];
            ++steps;
            if (record) store_state<S, K>(rec + (u64)(dd - 1) * NW, w, m);
            v = check_invariants<S, K>(w, m, P);
            if (v)
                atomicMin((unsigned long long*)&out->viol,
                          (unsigned long long)(((u64)dd << 44) | ((u64)(v - 1) << 40) | t));
        }
    }
    atomicAdd((unsigned long long*)&out->steps, (unsigned long long)steps);
    if (trunc) atomicAdd((unsigned long long*)&out->truncated, (unsigned long long)trunc);
    if (dead) atomicAdd((unsigned long long*)&out->deadlocked, (unsigned long long)dead);
}

template <int S, int K>
static hipError_t launch_sim_t(const Params& P, const u32* inits, u64 n_init, u64 n_beh, int depth, u64 seed,
                               int mode, SimCounters* out, i64 rec_beh, u32* rec, hipStream_t st) {
    const u64 blocks = (n_beh + 255) / 256;
    const u64 g = blocks < 4096 ? blocks : 4096;
    hipLaunchKernelGGL((k_simulate<S, K>), dim3((unsigned)g), dim3(256), 0, st, P, inits, n_init, n_beh, depth, seed,
                       mode, out, rec_beh, rec);
    return hipGetLastError();
}

// ---- host launchers (template dispatch on S, K, symmetry) ------------------------------
// Blocks of the expansion kernels (RMC_EXPAND_GRID for A/B runs; default
// 1024 = the resident blocks at 4 waves/SIMD: 4 per CU x 256 CUs, so a launch
// is one block round and every window sorts more tiles; 309.7 vs 315.6 ms per
// MCraftBench BFS against 2048, profiles/r03/ab/).  The other grid-stride
// kernels run 2048 blocks.
static u64 expand_grid_env() {
    static u64 v = [] {
        const char* e = getenv("RMC_EXPAND_GRID");
        const long long x = e ? atoll(e) : 0;
        return x >= 64 && x <= (1 << 20) ? (u64)x : (u64)0;
    }();
    return v;
}
// One round of resident blocks of kernel `k` on this device (blocks per CU at
// its register / LDS occupancy x CUs), cached per kernel and device: 1024 for
// the 4-wave sorted kernels, 1280 for the 5-wave every-lane kernel (a fixed
// 1024 left a fifth of the CUs' slots idle on S = 5: 0.339 s vs 0.289 s).
static u64 resident_grid(const void* k) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, u64> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({k, dev});
    if (it != cache.end()) return it->second;
    int nb = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 256, 0) != hipSuccess || nb <= 0) nb = 4;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const u64 v = (u64)nb * (u64)cus;
    cache[{k, dev}] = v;
    return v;
}

// Expansion kernel variant (RMC_EXPAND_VARIANT): 20 (the default, any value but 1)
// = k_expand_sort over windows of 16 tiles presorted by class (k_window_order; no
// sort in the kernel, so a smaller block), 5 probes in flight per thread, the
// parent's mixes recomputed per lane (80 VGPRs: 6 waves/SIMD; 5 waves for S >= 4), each wave taking its
// next quarter-window from a launch-wide counter (XL 739.3-741.6 vs 760.1-762.1 ms
// for fixed per-block shares, profiles/r05/variants/); 1 = every lane of every
// state (k_expand, the kernel of shapes with more than 128 lanes).  The variants
// measured and rejected in rounds 2-5 (6 probes at 5 waves with the mixes held,
// windows sorted in LDS, fixed shares, 4-8 probes at 4-6 waves, prefetching, 64-B
// store records) are in git history; their numbers are in DESIGN.md §Kernels.
static int expand_variant() {
    static int v = [] {
        const char* e = getenv("RMC_EXPAND_VARIANT");
        return e ? atoi(e) : 20;
    }();
    return v;
}

// Sharded expansion kernel (RMC_DIST_KVARIANT): 3 (the default, any value but 0)
// = the pool flush at the single-GPU kernel's shape (presorted windows, 5 probes,
// 6 waves/SIMD; remote successors pooled whole and routed by k_route after the
// launch); 0 = the round-3 send-marker kernel with the flush doing the routing
// (windows sorted in LDS).  The other variants measured in rounds 3-6
// (profiles/r04/ab/dist_kvariant_*, profiles/r05/kv4/; dynamic per-wave units a
// tie again in round 6, profiles/r06/ab/dist_kvariant_3_4.txt) are in git history.
static int dist_kvariant() {
    static int v = [] {
        const char* e = getenv("RMC_DIST_KVARIANT");
        return e ? atoi(e) : 3;
    }();
    return v;
}

// SYMMETRY expansion kernel (RMC_SYM_VARIANT): 2 (default) windows presorted by
// k_window_order, 6 probes in flight, 5 waves/SIMD (96 VGPRs, 28.7 KB of LDS:
// 79-80 ms on MCraftBenchSym, profiles/r06/ab/sym_batch6_5waves.txt); 1 the same
// with 8 probes at 4 waves (81-82 ms; dynamic per-wave units and other grids
// measured the same, profiles/r06/ab/sym_presorted.txt); 0 windows sorted in LDS
// by the kernel itself (round 5: 48 KB of LDS, 3 waves/SIMD, 87-88 ms).
static int sym_variant() {
    static int v = [] {
        const char* e = getenv("RMC_SYM_VARIANT");
        return e ? atoi(e) : 2;
    }();
    return v;
}

// Probes in flight per thread: 8 (measured best of 4/8/16 on MI355X).
constexpr int kBatch = 8;

template <int S, int K, bool SYM>
static hipError_t launch_t(int which, bool verify, const Params& P, const PermTable& PT, const DevBufs& B, u64 a,
                           u64 b, const u32* in, u32* out, u64 cap, unsigned long long* count, hipStream_t st) {
    const u64 n = (which == 0 || which == 3 || which == 5 || which == 7 || which == 12 || which == 13) ? (b - a)
                : which == 8 ? a * (u64)B.world : (which == 10 || which == 14) ? 1 : a;
    if (n == 0) return hipSuccess;
    const u64 blocks = (n + 255) / 256;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    // grid-stride kernels: 2048 blocks; the plain and sharded expansion kernels
    // one round of resident blocks (resident_grid at their launch below;
    // SYMMETRY keeps 2048: 79.7 vs 81.5 ms on the MCraftBench bounds)
    const u64 grid = (u64)2048;
    const u64 g = blocks < grid ? blocks : grid;
    // the expansion kernels' grid: RMC_EXPAND_GRID, else one round of resident blocks
    auto eg = [&](const void* k) -> unsigned {
        const u64 want = expand_grid_env() ? expand_grid_env() : resident_grid(k);
        return (unsigned)(blocks < want ? blocks : want);
    };
#define RMC_EXPAND_LAUNCH(KERNEL)                                                                              \
    hipLaunchKernelGGL(KERNEL, dim3(eg(reinterpret_cast<const void*>(&(KERNEL)))), dim3(256), 0, st, P, PT, B, a, b)
    constexpr bool SORTED = Lanes<S, K>::N <= 128;  // every shape: the lane-superset walk (LaneMask)
    if (which == 0) {
        if constexpr (SYM) {
            if (verify)
                hipLaunchKernelGGL((k_expand<S, K, true, kBatch, false, true>), dim3((unsigned)g), dim3(256), 0, st, P,
                                   PT, B, a, b);
            else if (sym_variant() >= 2 && S <= 3 && K == 4 && SORTED && B.word) {
                // presorted, 6 probes in flight, 5 waves/SIMD (the shapes that fit 96 VGPRs
                // without spills; the others take variant 1)
                if constexpr (S <= 3 && K == 4) {
                    const u64 gs = expand_grid_env() ? (blocks < expand_grid_env() ? blocks : expand_grid_env()) : g;
                    if (hipError_t e = launch_window_order(B, a, b, gs, 16, st)) return e;
                    hipLaunchKernelGGL((k_expand_sym<S, K, 6, SORTED, true, 0, 5>), dim3((unsigned)gs), dim3(256), 0,
                                       st, P, PT, B, a, b);
                }
            } else if (sym_variant() != 0 && SORTED && B.word) {  // windows presorted by k_window_order
                const u64 gs = expand_grid_env() ? (blocks < expand_grid_env() ? blocks : expand_grid_env()) : g;
                if (hipError_t e = launch_window_order(B, a, b, gs, 16, st)) return e;
                hipLaunchKernelGGL((k_expand_sym<S, K, kBatch, SORTED, true>), dim3((unsigned)gs), dim3(256), 0, st, P,
                                   PT, B, a, b);
            } else
                hipLaunchKernelGGL((k_expand_sym<S, K, kBatch, SORTED>), dim3((unsigned)g), dim3(256), 0, st, P, PT, B,
                                   a, b);
        } else if (verify) {
            RMC_EXPAND_LAUNCH((k_expand<S, K, false, kBatch, false, true>));
        } else if (expand_variant() != 1 && S >= 4 && SORTED && B.word) {
            // S >= 4 (68 / 92 lanes, the 128-bit lane mask): the same kernel at 5 waves/SIMD
            // (96 VGPRs, 16 B of scratch) beats 6 waves with 48 B of spills: MCraft5 -depth 20
            // 206 vs 245-246 ms (4 probes at 6 waves 247-248 ms), profiles/r06/ab/s5_waves.txt
            if constexpr (S >= 4) {
                const void* kp = reinterpret_cast<const void*>(&(k_expand_sort<S, K, 5, K <= 4 ? 1 : 0, true, 5, false, 1>));
                const u64 want = expand_grid_env() ? expand_grid_env() : resident_grid(kp);
                if (hipError_t e = launch_window_order(B, a, b, want, 16, st)) return e;
                RMC_EXPAND_LAUNCH((k_expand_sort<S, K, 5, K <= 4 ? 1 : 0, true, 5, false, 1>));
            }
        } else if (expand_variant() != 1 && S < 4 && SORTED && B.word) {  // 20: presorted windows, dynamic units
            if constexpr (S < 4) {
                const void* kp = reinterpret_cast<const void*>(&(k_expand_sort<S, K, 5, K <= 4 ? 1 : 0, true, 6, false, 1>));
                const u64 want = expand_grid_env() ? expand_grid_env() : resident_grid(kp);
                if (hipError_t e = launch_window_order(B, a, b, want, 16, st)) return e;
                RMC_EXPAND_LAUNCH((k_expand_sort<S, K, 5, K <= 4 ? 1 : 0, true, 6, false, 1>));
            }
        } else {  // 1, and shapes with more than 64 lanes
            RMC_EXPAND_LAUNCH((k_expand<S, K, false, kBatch, false, false, true>));
        }
    } else if (which == 3 && verify) {  // sharded full-state verification: every lane, hits compared
        RMC_EXPAND_LAUNCH((k_expand<S, K, SYM, kBatch, true, true>));
    } else if (which == 3) {
        if constexpr (SYM) RMC_EXPAND_LAUNCH((k_expand<S, K, SYM, kBatch, true>));  // the lossy sent-cache
        else if (dist_kvariant() != 0 && S >= 4 && B.pool) {
            // S >= 4: 5 waves/SIMD (96 VGPRs) instead of 6 with 96 B of spills: MCraft5 to
            // depth 20 on one sharded rank 0.322 vs 0.568 s (profiles/r06/ab/s5_dist_waves.txt)
            if constexpr (SORTED && S >= 4) {
                const void* kp = reinterpret_cast<const void*>(&(k_expand_dist<S, K, 5, false, true, 5, true>));
                const u64 want = expand_grid_env() ? expand_grid_env() : resident_grid(kp);
                if (hipError_t e = launch_window_order(B, a, b, want, 16, st)) return e;
                RMC_EXPAND_LAUNCH((k_expand_dist<S, K, 5, false, true, 5, true>));
            }
        } else if (dist_kvariant() != 0 && B.pool) {  // 3: the pool flush at the single-GPU kernel's shape
            if constexpr (SORTED && S < 4) {
                const void* kp = reinterpret_cast<const void*>(&(k_expand_dist<S, K, 5, false, true, 6, true>));
                const u64 want = expand_grid_env() ? expand_grid_env() : resident_grid(kp);
                if (hipError_t e = launch_window_order(B, a, b, want, 16, st)) return e;
                RMC_EXPAND_LAUNCH((k_expand_dist<S, K, 5, false, true, 6, true>));
            } else if constexpr (!SORTED) {
                RMC_EXPAND_LAUNCH((k_expand_dist<S, K, kBatch, false, false, 4, true>));
            }
        } else RMC_EXPAND_LAUNCH((k_expand_dist<S, K, kBatch, false>));            // send markers
    } else if (which == 12) {  // a replicated level: records [a, b) of B.rep (plain kernel, <= 64 lanes)
        if constexpr (!SYM && SORTED) RMC_EXPAND_LAUNCH((k_expand_dist<S, K, kBatch, true>));
        else return hipErrorInvalidValue;
    } else if (which == 14) {  // the pool's records to the outboxes (after a pool-flush expansion)
        if constexpr (!SYM) {
            hipLaunchKernelGGL((k_route_fix<S, K>), dim3(256), dim3(256), 0, st, P, B);
            hipLaunchKernelGGL((k_route<S, K>), dim3(1024), dim3(256), 0, st, P, B);
        } else {
            return hipErrorInvalidValue;
        }
    } else if (which == 13) {
        hipLaunchKernelGGL((k_pack_rep<S, K>), dim3((unsigned)g), dim3(256), 0, st, B, a, b, out);
    } else if (which == 11) {
        hipLaunchKernelGGL((k_compare_remote<S, K, SYM>), dim3((unsigned)g), dim3(256), 0, st, P, PT, B, in, a);
    } else if (which == 8) {  // a = keys per destination block (max); out = replies
        hipLaunchKernelGGL((k_materialize_remote<S, K>), dim3((unsigned)g), dim3(256), 0, st, P, B,
                           reinterpret_cast<const uint8_t*>(in), a, b);
    } else if (which == 9) {
        hipLaunchKernelGGL((k_store_remote<S, K>), dim3((unsigned)g), dim3(256), 0, st, P, B, in, a);
    } else if (which == 10) {
        if constexpr (SYM) hipLaunchKernelGGL((k_ties<S, K>), dim3(1024), dim3(256), 0, st, P, PT, B);
    } else if (which == 5) {
        hipLaunchKernelGGL((k_publish<S, K, SYM>), dim3((unsigned)g), dim3(256), 0, st, P, PT, B, a, b);
    } else if (which == 7) {
        hipLaunchKernelGGL((k_rehash<S, K, SYM>), dim3((unsigned)g), dim3(256), 0, st, P, PT, B, a, b);
    } else if (which == 6) {
        hipLaunchKernelGGL((k_verify<S, K, SYM>), dim3((unsigned)g), dim3(256), 0, st, P, PT, B, a);
    } else if (which == 15) {
        hipLaunchKernelGGL((k_verify_host<S, K, SYM>), dim3((unsigned)g), dim3(256), 0, st, P, PT, B, in, a, b);
    } else if (which == 1) {
        hipLaunchKernelGGL((k_seed<S, K, SYM>), dim3((unsigned)blocks), dim3(256), 0, st, P, PT, B, in, a);
    } else {
        hipLaunchKernelGGL((k_list<S, K, SYM>), dim3((unsigned)blocks), dim3(256), 0, st, P, PT, in, a, out, cap,
                           count);
    }
#undef RMC_EXPAND_LAUNCH
    if ((which == 0 || which == 3) && P.unbounded)  // depth-bounded unconstrained model: the capacity pass
        hipLaunchKernelGGL((k_capacity_check<S, K>), dim3((unsigned)g), dim3(256), 0, st, P, B, a, b);
    return hipGetLastError();
}

template <int S, int K>
static hipError_t launch_sk(bool sym, bool verify, int which, const Params& P, const PermTable& PT, const DevBufs& B,
                            u64 a, u64 b, const u32* in, u32* out, u64 cap, unsigned long long* count,
                            hipStream_t st) {
    if (sym) return launch_t<S, K, true>(which, verify, P, PT, B, a, b, in, out, cap, count, st);
    return launch_t<S, K, false>(which, verify, P, PT, B, a, b, in, out, cap, count, st);
}

// ---- objects: one per shape (RMC_SHAPE_S / RMC_SHAPE_K, the template
// instantiations, built in parallel) + the common object (dispatch, the
// shape-free kernels).  The fingerprint salt is a __constant__ of each object.
#define RMC_SHAPES(X) X(2, 4) X(2, 8) X(3, 4) X(3, 8) X(4, 4) X(4, 8) X(5, 4) X(5, 8)
#define RMC_SHAPE_DECLS(SS, KK)                                                                                 \
    hipError_t launch_shape_##SS##_##KK(const Shape& sh, int which, const Params& P, const PermTable& PT,       \
                                        const DevBufs& B, u64 a, u64 b, const u32* in, u32* out, u64 cap,       \
                                        unsigned long long* count, hipStream_t st);                             \
    hipError_t launch_sim_shape_##SS##_##KK(const Params& P, const u32* inits, u64 n_init, u64 n_beh, int depth, \
                                            u64 seed, int mode, SimCounters* out, i64 rec_beh, u32* rec,        \
                                            hipStream_t st);                                                    \
    hipError_t set_fp_salt_shape_##SS##_##KK(u64 salt, u64 ep, hipStream_t st);
RMC_SHAPES(RMC_SHAPE_DECLS)

#ifdef RMC_SHAPE_S
#define RMC_DEFINE_SHAPE(SS, KK)                                                                                \
    hipError_t launch_shape_##SS##_##KK(const Shape& sh, int which, const Params& P, const PermTable& PT,       \
                                        const DevBufs& B, u64 a, u64 b, const u32* in, u32* out, u64 cap,       \
                                        unsigned long long* count, hipStream_t st) {                            \
        return launch_sk<SS, KK>(sh.sym, sh.verify, which, P, PT, B, a, b, in, out, cap, count, st);           \
    }                                                                                                           \
    hipError_t launch_sim_shape_##SS##_##KK(const Params& P, const u32* inits, u64 n_init, u64 n_beh, int depth, \
                                            u64 seed, int mode, SimCounters* out, i64 rec_beh, u32* rec,        \
                                            hipStream_t st) {                                                   \
        return launch_sim_t<SS, KK>(P, inits, n_init, n_beh, depth, seed, mode, out, rec_beh, rec, st);        \
    }                                                                                                           \
    hipError_t set_fp_salt_shape_##SS##_##KK(u64 salt, u64 ep, hipStream_t st) {                                \
        /* staged on this call's stack and waited for: concurrent callers (one host */                          \
        /* thread per GPU in rmc-tlc -gpus N) share no staging buffer */                                        \
        const u64 h_salt = salt, h_ep = ep;                                                                     \
        hipError_t e =                                                                                          \
            hipMemcpyToSymbolAsync(HIP_SYMBOL(c_fp_salt), &h_salt, sizeof h_salt, 0, hipMemcpyHostToDevice, st); \
        if (e == hipSuccess)                                                                                    \
            e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_set_ep), &h_ep, sizeof h_ep, 0, hipMemcpyHostToDevice, st); \
        return e != hipSuccess ? e : hipStreamSynchronize(st);                                                  \
    }
#define RMC_DEFINE_SHAPE_(SS, KK) RMC_DEFINE_SHAPE(SS, KK)
RMC_DEFINE_SHAPE_(RMC_SHAPE_S, RMC_SHAPE_K)
#else


hipError_t set_fp_salt(const Shape& sh, u64 seed, u32 set_epoch, hipStream_t st) {
    const u64 salt = seed ? (mix64(seed) & ((1ull << 59) - 1)) : 0ull;
    if (set_epoch > 255) return hipErrorInvalidValue;
    const u64 ep = (u64)set_epoch << 56;
    // the common object's kernels insert too (k_owner_insert: sharded keys received)
    {
        const u64 h_ep = ep;
        const hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_set_ep), &h_ep, sizeof h_ep, 0, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) return e;
    }
    // only the ctx's shape object runs its kernels (the call waits for both copies)
#define RMC_SET_SALT(SS, KK) \
    if (sh.S == SS && sh.K == KK) return set_fp_salt_shape_##SS##_##KK(salt, ep, st);
    RMC_SHAPES(RMC_SET_SALT)
#undef RMC_SET_SALT
    return hipErrorInvalidValue;
}

hipError_t launch(const Shape& sh, int which, const Params& P, const PermTable& PT, const DevBufs& B, u64 a, u64 b,
                  const u32* in, u32* out, u64 cap, unsigned long long* count, hipStream_t st) {
#define RMC_CASE(SS, KK) \
    if (sh.S == SS && sh.K == KK) return launch_shape_##SS##_##KK(sh, which, P, PT, B, a, b, in, out, cap, count, st);
    RMC_SHAPES(RMC_CASE)
#undef RMC_CASE
    return hipErrorInvalidValue;
}

hipError_t launch_sim(const Shape& sh, const Params& P, const u32* inits, u64 n_init, u64 n_beh, int depth, u64 seed,
                      int mode, SimCounters* out, i64 rec_beh, u32* rec, hipStream_t st) {
#define RMC_SCASE(SS, KK) \
    if (sh.S == SS && sh.K == KK)   \
        return launch_sim_shape_##SS##_##KK(P, inits, n_init, n_beh, depth, seed, mode, out, rec_beh, rec, st);
    RMC_SHAPES(RMC_SCASE)
#undef RMC_SCASE
    return hipErrorInvalidValue;
}
#endif  // RMC_SHAPE_S

}  // namespace rmc
