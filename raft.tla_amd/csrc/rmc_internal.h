// rmc_internal.h — structures shared by the host engine and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "raft_packed.h"
#include "raft_wide.h"

namespace rmc {

// Device-side counters of one BFS level (zeroed/reset by the host per level).
struct Counters {
    u64 count;      // next free index of the state store (= distinct so far)
    u64 generated;  // successors generated in this launch
    u64 viol;       // min over violating new states of (index << 4 | invariant), ~0 = none
    u64 deadlock;   // min index of a state with no enabled lane, ~0 = none
    u32 overflow;   // state store full
    u32 table_full; // fingerprint set full
    u64 probes;     // fingerprint-set probes issued by k_expand
    // full-state verification mode (RMC_FLAG_VERIFY_STATES)
    u64 collisions; // fingerprint hits whose stored state differs from the successor
    u64 vchecked;   // fingerprint hits compared state against state
    u64 vcount;     // deferred hits in vbuf (stored twin not yet published)
    u64 nties;      // SYMMETRY: successors with tied signatures deferred to k_ties
    u64 novf;       // sharded: keys that did not fit their owner's outbox (parked in B.ovf)
    u64 wnext;      // dynamic work units: the next (window, wave slot) of the launch (zeroed by k_window_order)
    u64 walked;     // (state, lane) slots the lane walk visited (RMC_WALK_STATS: lane efficiency = generated / walked)
    u64 hcount;     // verification + spill: hits in hbuf whose stored owner has left the device window
};

struct DevBufs {
    u32* store;      // packed states, (2S + K) words each; levels are contiguous ranges
    u64* parent;     // parent index per state (~0 for initial states)
    uint8_t* act;    // lane that produced the state (255 for initial states)
    u64* foot;       // messages the producing lane acted on / added (make_foot; 0 = unknown)
    uint8_t* cls;    // window-sort class of each state (state_class_fine; a layout hint)
    uint16_t* word;  // presorted windows (k_window_order): the launch's window positions in class order
    u64* table;      // fingerprint set, power-of-two slots, 0 = empty
    u64 tmask;       // slots - 1
    u64 cap;         // state store capacity
    // ring window (RMC_FLAG_SPILL with the trace links in HBM): store / foot / cls hold
    // state i at slot i & wmask, the last wmask + 1 states; ~0 (resident, host-link
    // spill, sharded): slot = index.  parent / act are indexed by the index itself.
    u64 wmask;
    Counters* ctr;
    // sharded mode (rank/world > 1 GPU processes; single mode: rank 0, world 1)
    u32 rank, world;
    u32 owner_mode;            // 0: by fingerprint, 1: by server 0 word, 2: by servers 0+1 words (default), 3: all words
    u64 ref_tag;               // (rank << 48): parent refs are global (rank, index)
    u64* sent;                 // lossy cache of fingerprints already shipped to their owner
    u64 smask;                 // sent-cache slots - 1
    // two-phase exchange: phase 1 keys, phase 2 accepted states
    u64* key_out;              // [world][kcap] 12-B keys for each owner: the raw fingerprint {k lo, k hi, s32}
    u64* tick_out;             // [world][kcap] local tickets: parent index | lane << 56, or POOL_TICK | pool index
    u64 kcap;                  // keys per destination and chunk
    unsigned long long* ocount;  // [world] keys written per destination
    u32* st_out;               // [world][scap][NW + 4] accepted states for each owner (+ ref, footprint)
    u64 scap;                  // state records per destination and round (= kcap)
    unsigned long long* scount;  // [world] state records written per destination
    // keys whose owner's outbox was full: {k, s32 | flags << 32, parent index | dest << 48 |
    // lane << 56}, sent in later exchange rounds of the same level (never dropped);
    // flag OVF_UNKEYED: a successor the expansion could not put in the pool, keyed by k_route_fix
    u64* ovf;
    u64 ovf_cap;               // records in ovf
    // remote-successor pool (the sharded expansion's default flush, flush_pool):
    // every new successor owned by another rank, materialised once as its
    // phase-2 record {state, global parent ref | lane << 40, footprint}; k_route
    // then keys it and fills the owners' outboxes with tickets POOL_TICK | index
    u32* pool;
    u64 pool_cap;              // records in pool
    unsigned long long* npool; // records written (may exceed pool_cap: the rest were parked)
    // replicated levels (small levels of a sharded search): the whole level's
    // records, gathered from every rank (RepRec: state, global ref, footprint, lane | class)
    const u32* rep;
    // full-state verification mode: store index of the state owning each
    // fingerprint-set slot (~0 = not yet published; published between launches
    // by k_publish) and the deferred hits {parent index, slot | lane << 56}
    u64* sidx;
    u64* vbuf;
    u64 vcap;                  // records in vbuf
    // verification + spill: owners with a store index below vlo are no longer on
    // the device (spilled; their host copies are compared after the launch): such
    // hits go to hbuf as {parent index, owner index | lane << 56}
    u64 vlo;
    u64* hbuf;
    u64 hcap;                  // records in hbuf
    // SYMMETRY: successors whose server signatures tie, {parent index | lane << 56},
    // canonicalised by k_ties after each expansion launch
    u64* ties;
    u64 tie_cap;
};

struct PermTable {
    u32 code[120];  // every server permutation (old id -> new id), 3 bits per id, S <= 5
    int np;         // S!
};

struct Shape {
    int S, K;
    bool sym;
    bool verify;  // full-state verification (single GPU)
};

// which: 0 = k_expand over store[a, b); 1 = k_seed of `a` staged states `in`;
//        2 = k_list of `a` states `in` into `out` (cap records, *count);
//        3 = sharded k_expand over store[a, b) (outbox in B);
//        8 = k_materialize_remote of window [b, b + a) of each destination's keys, in = replies;
//        9 = k_store_remote of `a` received state records `in`;
//       10 = k_ties over the deferred tied successors (count on the device);
//        5 = k_publish over store[a, b) (verification: slot -> store index);
//        6 = k_verify of `a` deferred hits in B.vbuf;
//        7 = k_rehash of the stored states [a, b) (recovery).
//       11 = k_compare_remote of `a` received state records `in` (sharded verification);
//       12 = k_expand_dist<REP> over the replicated level's records B.rep[a, b);
//       13 = k_pack_rep of this rank's stored states [a, b) into records at `out`;
//       14 = k_route: key the pool's records and fill the outboxes (counts on the device);
//       15 = k_verify_host of `a` hits B.hbuf[b, b + a) against their owners' host copies
//            staged at `in` (verification + spill).
hipError_t launch(const Shape& sh, int which, const Params& P, const PermTable& PT, const DevBufs& B, u64 a, u64 b,
                  const u32* in, u32* out, u64 cap, unsigned long long* count, hipStream_t st);

// Simulation counters (k_simulate).
typedef int64_t i64;
struct SimCounters {
    u64 steps, truncated, deadlocked;
    u64 viol;  // min over violations of (depth << 44 | invariant << 40 | behaviour), ~0 = none
};
hipError_t launch_sim(const Shape& sh, const Params& P, const u32* inits, u64 n_init, u64 n_beh, int depth, u64 seed,
                      int mode, SimCounters* out, i64 rec_beh, u32* rec, hipStream_t st);

// Sharded mode, phase 1 owner side: insert n received keys (12-B {k lo, k hi, s32}
// records), reply[t] = new;
// keys [src_off[p], src_off[p + 1]) came from rank p, acc[p] += keys of p that were new.
constexpr int kMaxWorld = 64;
struct SrcOff {
    u64 o[kMaxWorld + 1];
};
hipError_t launch_owner_insert(const DevBufs& B, const u64* keys, uint8_t* reply, u64 n, const SrcOff& so,
                               unsigned long long* acc, hipStream_t st);
// Sharded mode: the exchange-count row of one round, one block of kRowWords u64
// per rank p: [0] keys for p (min(ocount[p], kcap), 0 for p = rank), [1] flags
// (bit 0: this rank has more to send: host_more, or parked keys beyond
// ovf_done; bit 1: its parking buffer overflowed; bit 2: it sends keys this
// round), [2..] this rank's Counters (so a round after which nothing changes
// them ends the level without a counter all-gather); out[kRowWords * W] = novf.
constexpr int kRowWords = 2 + (int)(sizeof(Counters) / 8);
static_assert(sizeof(Counters) % 8 == 0, "Counters travel as u64 words");
// mirror (a world of one): the row's blocks also written there (its received half).
hipError_t launch_pack_counts(const DevBufs& B, u64 host_more, u64 ovf_done, u64* out, hipStream_t st,
                              u64* mirror = nullptr);
// States per single-GPU expansion launch at most (B.word holds one launch's
// presorted window positions).
constexpr int kMaxLaunchLog2 = 25;
// Presorted windows: k_window_order over the launch [lo, hi) for an expansion
// grid of `grid` blocks and windows of at most wt_max tiles (B.word).
hipError_t launch_window_order(const DevBufs& B, u64 lo, u64 hi, u64 grid, u64 wt_max, hipStream_t st);
// The slot of state index i in the store / foot / cls arrays (DevBufs.wmask).
__host__ __device__ __forceinline__ u64 wslot(const DevBufs& B, u64 i) { return i & B.wmask; }
// Sharded mode: move parked keys ovf[a, a + n) into the (emptied) outbox; n <= kcap.
hipError_t launch_drain(const DevBufs& B, u64 a, u64 n, hipStream_t st);
// Outbox ticket of a pool record (bit 48: a parent ticket's index is < 2^48 and
// its lane sits at bits 56-63).
constexpr u64 POOL_TICK = 1ull << 48;

// Fingerprint salt for the kernels of shape sh on this device (0 = default
// hash); returns after the copy (the staging value lives on the caller's stack).
// the fingerprint salt of rmc_config.seed and the set epoch of the run (raft_packed.h
// c_set_ep: 0 = an untagged set, cleared before the run)
hipError_t set_fp_salt(const Shape& sh, u64 seed, u32 set_epoch, hipStream_t st);

// Sets bytes [p, p + bytes) to `byte` (the fingerprint set's clear; RMC_FILL=0: hipMemsetAsync).
hipError_t launch_fill(void* p, u64 bytes, uint8_t byte, hipStream_t st);
// Random-probe microbenchmark over table[mask + 1] (mode 0 loads, 1 CAS).
hipError_t launch_probe_bench(u64* table, u64 mask, u64 threads, u32 iters, int mode, u64* sink, hipStream_t st);

// ---- the wide layout (raft_wide.h, rmc_wide.hip) ------------------------------------
namespace wide {
struct WideBufs {
    void* store;      // wide records (WState, WStateC or WStateD); levels are contiguous ranges
    int compact;      // the store's record: 0 WState, 1 the compact WStateC, 2 the depth-sized WStateD
    u64* parent;      // parent index per state (~0 for initial states)
    uint8_t* act;     // lane that produced the state (255 for initial states)
    u64* table;       // fingerprint set (wfp keys), power-of-two slots
    u64 tmask, cap;
    Counters* ctr;
    u64 salt;         // fingerprint salt (rmc_config.seed)
};
// One successor listed by k_wlist (rmc_expand on the wide layout).
struct WSucc {
    u64 parent;
    int lane, code, in_model, pad;
    u64 fp;
    WState state;
};
hipError_t launch_wseed(const WModel& M, const WideBufs& B, const void* staged, u64 n, hipStream_t st);  // B's layout
hipError_t launch_wexpand(const WModel& M, const WideBufs& B, u64 lo, u64 hi, hipStream_t st);
hipError_t launch_wlist(const WModel& M, const WState* in, u64 n, WSucc* out, u64 cap, unsigned long long* count,
                        u64 salt, hipStream_t st);
hipError_t launch_wsimulate(const WModel& M, const WState* inits, u64 n_init, u64 n_beh, int depth, u64 seed, int mode,
                            SimCounters* out, i64 rec_beh, WState* rec, hipStream_t st);
}  // namespace wide

}  // namespace rmc
