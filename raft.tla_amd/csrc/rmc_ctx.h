// rmc_ctx.h — the host-side context behind the C ABI (rmc_api.cpp, rmc_dist.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/rmc.h"
#include "raft_packed.h"
#include "rmc_internal.h"

// Sharded mode (rmc_shard): this ctx is one rank of a BFS whose fingerprint
// space is partitioned over `world` GPUs.  The exchange runs
// over RCCL (one communicator per ctx, on the ctx stream) or over a
// caller-supplied host transport (rmc_transport, e.g. gloo in tests).
struct DistState {
    int on = 0;
    int rank = 0, world = 1;
    int rccl = 0;                   // 1: RCCL communicator, 0: host transport
    ncclComm_t comm = nullptr;
    rmc_transport host{};
    hipStream_t xs = nullptr;       // exchange stream: every collective, owner insert, phase 2
    // Outbox sets, double-buffered: the expansion of round k + 1 (ctx stream)
    // fills one set while round k's exchange (xs) drains the other.
    struct Set {
        rmc::u64* key_out = nullptr;             // [world][kcap] 12-B keys per owner {k lo, k hi, s32}
        rmc::u64* tick_out = nullptr;            // [world][kcap] tickets (parent | lane << 56)
        unsigned long long* ocount = nullptr;    // [world] keys written per owner, [world]: pool records
        rmc::u32* pool = nullptr;                // remote-successor pool (phase-2 records, flush_pool)
        rmc::u64* cx = nullptr;                  // device count row: [2W + 1] sent, [2W] received
        rmc::u64* h_cx = nullptr;                // pinned copy of cx
        hipEvent_t ev_exp = nullptr;             // expansion (or drain) of this set's round done
        hipEvent_t ev_free = nullptr;            // the round's exchange no longer reads the set
        hipEvent_t k0 = nullptr, k1 = nullptr;   // expansion kernel time
        hipEvent_t x0 = nullptr, x1 = nullptr;   // exchange time (xs) of the round
        int timed = 0, xtimed = 0;
    } set[2];
    hipEvent_t ev_cnt = nullptr, ev_acc = nullptr, ev_c = nullptr, ev_x = nullptr;
    hipEvent_t ev_h = nullptr;      // host waits on xs (under the deadline)
    // single buffers (used on xs only, rounds in order)
    rmc::u64* key_in = nullptr;     // keys received (12-B {k, s32} records), blocks by source
    uint8_t* rep_out = nullptr;     // replies to the keys received (same layout)
    uint8_t* rep_in = nullptr;      // replies to the keys sent, [world][kcap]
    rmc::u32* st_in = nullptr;      // accepted states received, blocks by source
    unsigned long long* sa = nullptr;  // [2W]: states to send per owner (scount), states to receive per source
    rmc::u64* h_sa = nullptr;       // pinned copy of sa
    rmc::u64 in_cap = 0;            // keys / states receivable per round (all sources)
    void* ag_dev = nullptr;         // RCCL all-gathers of small rows: device staging,
    rmc::u64 ag_cap = 0;            // (world + 1) x ag_cap bytes, allocated once per shard
    std::vector<uint8_t> stage_send, stage_recv;  // host transport staging
    rmc::u64 sent_slots = 0;
    rmc::u64 pool_cap = 0;          // records per pool (one pool per outbox set)
    int debug = 0;                  // RMC_DIST_DEBUG: one stderr line per round
    int table_grown = 0;            // rmc_shard doubled the fingerprint set once (send markers)
    int split = 2;                  // RMC_DIST_SPLIT: rounds a large level is cut into at least (1 at world 1)
    int overlap = 1;                // RMC_DIST_OVERLAP=0: the next expansion waits for the exchange
    double fill = 0.5;              // RMC_DIST_FILL: expected fill of the fullest outbox a round aims at
                                    // (> 1 forces parking: a test hook)
    // replicated levels: a level of at most rep_max states in total is gathered
    // whole (k_pack_rep records) into rep_buf on every rank and expanded there
    rmc::u64 rep_max = 0;
    rmc::u32* rep_send = nullptr;   // this rank's records of the level
    rmc::u32* rep_buf = nullptr;    // every rank's, in rank order
    rmc::u64 rep_levels = 0;        // replicated levels of the last run
    // deadlines (RMC_DIST_TIMEOUT_S) and where the loop is, for error messages
    double timeout_s = 300.0;
    int nonblocking = 0;            // the RCCL communicator is non-blocking
    int aborted = 0;                // a deadline aborted the communicator: the ctx is unusable
    int abort_pending = 0;          // ... and the abort has not returned: device buffers are leaked, not freed
    int lvl = 0, rnd = 0;
    const char* phase = "";
    int stall_rank = -1, stall_level = 2;  // test hook (RMC_DIST_STALL_*)
    double stall_s = 0;
    // statistics of the last run
    rmc::u64 keys_sent = 0, states_sent = 0, chunks = 0, parked = 0;
    double xfer_seconds = 0;        // device time of the exchange rounds (xs), overlapped or not
    double wait_seconds = 0;        // host wall time blocked on count read-backs and level ends
};

// Frontier spill (RMC_FLAG_SPILL): the device holds the fingerprint set and
// the window of states [base, base + win) — the frontier being expanded and the
// level being built.  Below base only the trace links survive, in host memory:
// parent index + action lane per state (9 B, TLC's trace file), and a
// counterexample re-derives those states by replaying the lanes from Init.
// B.store / B.parent / B.act are biased by -base, so kernels keep indexing
// states by their global index.
struct SpillState {
    int on = 0;
    // device links (default when they fit): the trace links of every state stay in
    // HBM (9 B per state, B.parent / B.act indexed by global index, never rebased)
    // and a spill only shifts the window's states, footprints and classes — no
    // PCIe traffic; otherwise (RMC_SPILL_HOST_LINKS=1, or no room) they move to
    // the host as below
    int dev_links = 0;
    rmc::u64 base = 0;          // first device-resident global index
    rmc::u64 win = 0;           // device window (states)
    rmc::u64 total_cap = 0;     // all states (fingerprint-set sizing)
    rmc::u32* store = nullptr;  // the real device allocations
    rmc::u64* parent = nullptr;
    uint8_t* act = nullptr;
    rmc::u64* foot = nullptr;
    uint8_t* cls = nullptr;
    rmc::u64* h_parent = nullptr;  // host, [total_cap], reserved address space,
    uint8_t* h_act = nullptr;      // pages touched as levels spill
    size_t h_bytes = 0;
    rmc::u64 faulted = 0;          // links [0, faulted) have backed pages
    std::thread ahead;             // backs the next window's pages during expansion
    // verification + spill (RMC_FLAG_VERIFY_STATES): a host copy of every state that
    // leaves the device window ([0, hcopied) copied), against which the hits on
    // spilled owners are checked (B.hbuf, k_verify_host); reserved like the links
    rmc::u32* h_state = nullptr;
    size_t hs_bytes = 0;
    rmc::u64 hcopied = 0;
    rmc::u32* h_ostage = nullptr;  // pinned / device staging of the owners of one batch of hits
    rmc::u32* d_ostage = nullptr;
    rmc::u64 ostage_cap = 0;       // states per batch
    rmc::u64 host_hits = 0;        // hits checked against host copies in the last run
};

// rmc_config.set_bytes -> fingerprint-set slots: the largest power of two of
// 8-B slots within the bytes (at least 1024), 0 when the set is sized automatically
inline rmc::u64 set_slots_of(rmc::u64 bytes) {
    if (bytes == 0) return 0;
    rmc::u64 sl = 1024;
    while ((sl << 1) * 8 <= bytes) sl <<= 1;
    return sl;
}

struct rmc_ctx {
    rmc_config cfg{};
    rmc::Shape sh{};
    rmc::Params P{};
    rmc::PermTable PT{};
    int NW = 0;  // 32-bit words per packed state
    hipStream_t st = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;  // bracket each level's expansion launches
    rmc::DevBufs B{};
    rmc::Counters* h_ctr = nullptr;  // pinned
    rmc::u32* d_staged = nullptr;
    rmc::u64 table_slots = 0;
    // the epoch the set's current entries carry (raft_packed.h c_set_ep): 0 = untagged
    // (cleared to 0 by the last run, or unknown), 1..255 = tagged; the next plain
    // single-GPU run takes the next epoch without clearing the set (rmc_run_bfs)
    rmc::u32 set_epoch = 0;
    rmc::u64 walked = 0;  // (state, lane) slots of the lane walk in the last run (RMC_WALK_STATS)
    rmc_result res{};
    std::string err;
    std::vector<rmc::u64> level_start;  // level d (1-based) = [level_start[d-1], level_start[d])
    int have_target = 0;                // a violation / deadlock state to trace
    rmc::u64 target_idx = 0;            // sharded: global ref (rank << 48 | index)
    DistState dist;
    SpillState spill;
    // recovery (rmc_recover): the next rmc_run_bfs continues from this level
    int resume = 0;
    int resume_depth = 0;
    // the wide layout (raft_wide.h): bounds beyond the packed capacity
    int wide = 0;
    rmc::wide::WModel WM{};
    rmc::wide::WideBufs WB{};
    rmc::wide::WState* w_staged = nullptr;
};

#define HIPCHK(c, expr)                                                                              \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess)                                                                        \
            return rmc_host::fail((c), e_ == hipErrorOutOfMemory ? RMC_E_NOMEM : RMC_E_HIP,           \
                                  std::string(#expr) + ": " + hipGetErrorString(e_));                \
    } while (0)

namespace rmc_host {
// TLC's "calculated (optimistic)" collision estimate D * (G - D) / 2^b for the
// fingerprint bits b the set compares: 64 of k plus the bits of the second sum
// folded in under the slot mask, min(32, log2 slots) (raft_packed.h Fp).
inline double fp_collision_estimate(double D, double G, rmc::u64 slots, bool tagged = false) {
    int lb = 0;
    while (lb < 32 && (2ull << lb) <= slots) ++lb;
    // a tagged set compares 56 + lb bits (the top 8 hold the run's epoch)
    return D * (G - D) / 18446744073709551616.0 / (double)(1ull << lb) * (tagged ? 256.0 : 1.0);
}
int fail(rmc_ctx* c, int code, const std::string& msg);
int kcap_for(int max_msgs);
int validate(const rmc_config* c, std::string* why);
void fill_params(rmc_ctx* c);
int family_of(const rmc::Params& P, int lane);
int encode_view(const rmc_ctx* c, const rmc_state_view& v, rmc::u32* out, std::string* why);
void decode_state(const rmc_ctx* c, const rmc::u32* in, rmc_state_view* v);
void init_view(const rmc_config& g, rmc_state_view* v);
int reset_counters(rmc_ctx* c, bool keep_count);
int read_counters(rmc_ctx* c);
// RMC_E_CAPACITY message for an unbounded field a successor took past the
// packed capacity (Counters.overflow bits 8-11), "" if none
std::string capacity_message(const rmc_ctx* c, rmc::u32 overflow, int depth);
// sharded mode (rmc_dist.cpp)
int run_bfs_sharded(rmc_ctx* c, rmc_progress_fn cb, void* user);
int trace_sharded(rmc_ctx* c, rmc_state_view* states, int32_t* families, int32_t* instances, size_t cap,
                  size_t* len);
void free_dist(rmc_ctx* c);
// frontier spill (rmc_api.cpp)
void spill_rebase(rmc_ctx* c, rmc::u64 base);
int spill_reserve(rmc_ctx* c);
int spill_to(rmc_ctx* c, rmc::u64 a, rmc::u64 count);
void spill_free(rmc_ctx* c);
int read_link(rmc_ctx* c, rmc::u64 idx, rmc::u64* parent, uint8_t* act);
// the wide layout (rmc_wide.cpp)
bool wide_wanted(const rmc_config& g);
size_t wide_record_bytes(const rmc_config& g);  // the BFS store's record: compact or full
int validate_wide(const rmc_config* c, std::string* why);
int create_wide(rmc_ctx* c);
void destroy_wide(rmc_ctx* c);
int run_bfs_wide(rmc_ctx* c, rmc_progress_fn cb, void* user);
int trace_wide(rmc_ctx* c, rmc_state_view* states, int32_t* families, int32_t* instances, size_t cap, size_t* len);
int expand_wide(rmc_ctx* c, const rmc_state_view* states, size_t n, rmc_succ_view* out, size_t cap, size_t* n_out);
int sim_wide(rmc_ctx* c, const rmc_sim_config* sc, rmc_sim_result* out, rmc::i64 rec_beh,
             std::vector<rmc_state_view>* rec);
void fill_wide_model(rmc_ctx* c);
int smoke_views(const rmc_ctx* c, const rmc_sim_config& sc, std::vector<rmc_state_view>* views, std::string* why);
}  // namespace rmc_host
