/*
 * rmc.h — C ABI of librmc.so, the MI355X-native breadth-first model checker
 * for raft.tla (the hot path of TLC's `tlc2.TLC -config MCraft.cfg MCraft.tla`).
 *
 * The reference path has no FFI of its own: it sits behind TLC's CLI and file
 * formats.  Each entry point below replaces one piece of that
 * path; the reference interface it replaces is cited next to it.  A Java
 * driver binds these through Panama FFM; the C++ CLI
 * (`bin/rmc-tlc`) and the Python ctypes harness (tests, bench) bind the same
 * symbols.
 *
 * Conventions: plain C types only; return 0 on success and a negative code
 * otherwise (RMC_E_*); the message is available from rmc_last_error(ctx).
 * No C++ exception crosses the ABI.  A ctx owns all device memory; output
 * buffers are caller-owned.  Calls on one ctx are not reentrant.
 */
#ifndef RMC_H_
#define RMC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMC_ABI_VERSION 8 /* 6: rmc_result.spill_links_on_device (round 5); 7: .verified_spilled, 8: rmc_config.set_bytes and
                             rmc_result.set_slots (round 6) */

/* Capacity of the packed encoding (DESIGN.md "Packed state"): the layout the
 * BFS kernels run on when every bound fits it. */
#define RMC_MAX_SERVERS 5
#define RMC_MAX_VALUES 2
#define RMC_MAX_LOG 3      /* MaxLogLen bound <= 3 */
#define RMC_MAX_MSGS 8     /* |DOMAIN messages| bound <= 8 */
#define RMC_MAX_TERM 14    /* MaxTerm bound <= 14 */
#define RMC_MAX_DUP 3      /* per-message count bound <= 3 */
/* Capacity of the wide encoding (DESIGN.md "Wide state"): a model with any
 * bound beyond the packed capacity — or a field no CONSTRAINT bounds, under a
 * depth bound or in simulation — runs on it (single GPU; no SYMMETRY,
 * verification or spill).  A CONSTRAINT bound must stay below the wide
 * capacity; an unbounded field is given the capacity itself, and a successor
 * beyond it stops the search with RMC_E_CAPACITY naming the field. */
#define RMC_WIDE_MAX_TERM 255
#define RMC_WIDE_MAX_LOG 32
#define RMC_WIDE_MAX_MSGS 64
#define RMC_WIDE_MAX_DUP 255
/* Sizes of the decoded state view (rmc_state_view): the wide capacity. */
#define RMC_VIEW_LOG 32
#define RMC_VIEW_MSGS 64

/* Error codes. */
#define RMC_OK 0
#define RMC_E_INVAL (-22)      /* config validation failed (TLC: semantic error) */
#define RMC_E_NOMEM (-12)      /* device allocation failed */
#define RMC_E_HIP (-5)         /* HIP runtime error */
#define RMC_E_CAPACITY (-28)   /* fingerprint set full, or state store full without RMC_FLAG_SPILL */
#define RMC_E_NOGPU (-19)      /* no usable gfx950 device */
#define RMC_E_PARSE (-74)      /* .cfg / .tla front-end could not recognise the model */
#define RMC_E_STATE (-71)      /* call out of order (e.g. rmc_trace before a violation) */
#define RMC_E_IO (-61)         /* checkpoint file missing, unreadable or of another model */

/* rmc_config.flags */
#define RMC_FLAG_SYMMETRY (1u << 0)        /* SYMMETRY Permutations(Server)            */
#define RMC_FLAG_CHECK_DEADLOCK (1u << 1)  /* CHECK_DEADLOCK TRUE (TLC default)         */
#define RMC_FLAG_BUG_QUORUM (1u << 2)      /* BecomeLeader guard raft.tla:197 weakened  */
                                           /* to votesGranted[i] /= {} (config 5)       */
#define RMC_FLAG_VERIFY_STATES (1u << 3)   /* full-state verification: every fingerprint */
                                           /* hit is compared with the stored state;    */
                                           /* differences = collisions (no TLC analog;  */
                                           /* single GPU)                               */
#define RMC_FLAG_SPILL (1u << 4)           /* frontier spill (TLC's states/ directory): */
                                           /* expanded levels leave the device window   */
                                           /* when it fills, so a model whose states    */
                                           /* outgrow HBM completes while its           */
                                           /* fingerprints fit.  Their trace links      */
                                           /* (parent, lane: 9 B) stay in HBM when they */
                                           /* fit (else they move to host memory).      */
                                           /* state_capacity then sizes the fingerprint */
                                           /* set and links (all states), device_window */
                                           /* the resident states.  Single GPU.  With   */
                                           /* RMC_FLAG_VERIFY_STATES every state leaving */
                                           /* the window keeps a host copy, and hits on  */
                                           /* it are compared with that copy (round 6;   */
                                           /* no checkpoint / recover then)             */
/* A model without a CONSTRAINT on some field (MCraft.cfg as shipped) runs only
 * under a depth bound (max_depth > 0, TLC -depth).  The front-end then gives
 * each unbounded field the wide capacity (RMC_WIDE_MAX_TERM, RMC_WIDE_MAX_LOG,
 * RMC_WIDE_MAX_MSGS, RMC_WIDE_MAX_DUP) and sets its bit here; the search stops
 * with RMC_E_CAPACITY, naming the field, the first time a successor needs more
 * than the capacity (it is never silently filtered as out of the model). */
#define RMC_FLAG_UNBOUNDED_TERM (1u << 5)  /* no CONSTRAINT on currentTerm[i]            */
#define RMC_FLAG_UNBOUNDED_LOG (1u << 6)   /* no CONSTRAINT on Len(log[i])               */
#define RMC_FLAG_UNBOUNDED_MSGS (1u << 7)  /* no CONSTRAINT on Cardinality(DOMAIN messages) */
#define RMC_FLAG_UNBOUNDED_DUP (1u << 8)   /* no CONSTRAINT on messages[m]               */
#define RMC_UNBOUNDED_ANY (RMC_FLAG_UNBOUNDED_TERM | RMC_FLAG_UNBOUNDED_LOG | RMC_FLAG_UNBOUNDED_MSGS | \
                           RMC_FLAG_UNBOUNDED_DUP)

/* rmc_config.invariants — the INVARIANT names the engine knows (fused checks). */
#define RMC_INV_TYPEOK (1u << 0)           /* raft.tla:482-492                          */
#define RMC_INV_ONE_LEADER (1u << 1)       /* ElectionSafety restated (raft.tla:1124)   */
#define RMC_INV_LOG_MATCHING (1u << 2)     /* raft.tla:1132-1136                        */
#define RMC_INV_MESSAGES (1u << 3)         /* MessagesInv raft.tla:941-946 (:910 fixed)  */
#define RMC_INV_LEADER_VOTES (1u << 4)     /* LeaderVotesQuorum raft.tla:1033-1037       */
#define RMC_INV_CAND_TERM (1u << 5)        /* CandidateTermNotInLog raft.tla:1041-1047   */
/* The IsPrefix invariants (raft.tla:1143-1180), restated in specs/MCraftBounded.tla
 * with IsPrefix defined and Committed(i) = the first min(commitIndex[i], Len(log[i]))
 * entries of log[i] (raft.tla's SubSeq is out of range when commitIndex > Len). */
#define RMC_INV_VOTES_GRANTED (1u << 6)    /* VotesGrantedInv raft.tla:1145-1153         */
#define RMC_INV_QUORUM_LOG (1u << 7)       /* QuorumLogInv raft.tla:1157-1161            */
#define RMC_INV_MORE_UP_TO_DATE (1u << 8)  /* MoreUpToDateCorrect raft.tla:1167-1172     */
#define RMC_INV_LEADER_COMPLETE (1u << 9)  /* LeaderCompleteness raft.tla:1176-1180      */

/* A bounded model: constants of the MC module + the CONSTRAINT bounds.
 * Replaces the CONSTANTS / CONSTRAINT / INVARIANT / SYMMETRY / CHECK_DEADLOCK
 * sections of a TLC .cfg (MCraft.cfg:1-39, Smokeraft.cfg:43-48). */
typedef struct rmc_config {
    int32_t n_servers;        /* |Server|  (MCraft.tla:20-21: {r1,r2,r3})        */
    int32_t n_values;         /* |Value|   (MCraft.tla:15-16: {v1,v2})           */
    int32_t max_term;         /* CONSTRAINT \A i: currentTerm[i] <= max_term      */
    int32_t max_log_len;      /* CONSTRAINT \A i: Len(log[i]) <= max_log_len      */
    int32_t max_msgs;         /* CONSTRAINT Cardinality(DOMAIN messages) <= ..    */
    int32_t max_dup;          /* CONSTRAINT \A m: messages[m] <= max_dup          */
    uint32_t flags;           /* RMC_FLAG_*                                       */
    uint32_t invariants;      /* RMC_INV_*                                        */
    int32_t device;           /* HIP device ordinal                               */
    int32_t max_depth;        /* 0 = unbounded; else stop after this many levels  */
    uint64_t state_capacity;  /* distinct states this GPU may store; 0 = auto     */
    uint64_t seed;            /* BFS: fingerprint salt (0 = default hash; two runs */
                              /* with different salts and equal counts rule out   */
                              /* fingerprint collisions); simulation: RNG seed     */
    uint64_t device_window;   /* RMC_FLAG_SPILL: states resident on the device    */
                              /* (frontier + the level being built); 0 = auto     */
    uint64_t set_bytes;       /* the fingerprint set's size (TLC -fpmem), rounded */
                              /* down to a power of two of 8-B slots; it holds at */
                              /* most half as many states (a capacity error past  */
                              /* that).  With state_capacity given it is an upper */
                              /* bound, halved until the store fits beside it.    */
                              /* 0 = auto: 2 slots per state of state_capacity    */
                              /* (auto: for the largest store the device holds)   */
} rmc_config;

/* End-of-run summary.  Replaces TLC's stdout summary lines:
 * "N states generated, M distinct states found, Q states left on queue." and
 * "The depth of the complete state graph search is D." */
typedef struct rmc_result {
    uint64_t generated;        /* init states + every successor of every expanded state */
    uint64_t distinct;         /* distinct (canonical) states found                     */
    uint64_t left_on_queue;    /* frontier states not expanded at stop                  */
    int32_t depth;             /* BFS levels (init = level 1)                           */
    int32_t violated_inv;      /* RMC_INV_* bit of the violated invariant, or 0         */
    int32_t violation_depth;   /* level of the violating state, or 0                    */
    int32_t deadlock;          /* 1 if a state without successors was found             */
    double collision_probability; /* fingerprint collision estimate (TLC prints one too) */
    double seconds;            /* wall time of rmc_run_bfs                              */
    double expand_kernel_seconds; /* device time of the expansion kernels, HIP events on */
                                  /* the ctx stream (sum over levels)                    */
    uint64_t expand_launches;  /* expansion kernel launches (levels are split in chunks) */
    uint64_t probes;           /* fingerprint-set probes (successors that reached the set) */
    uint64_t collisions;       /* RMC_FLAG_VERIFY_STATES: fingerprint hits whose stored state */
                               /* differs (0 = the counts are exact, not probabilistic)   */
    uint64_t verified;         /* RMC_FLAG_VERIFY_STATES: hits compared state by state    */
    /* sharded mode (rmc_shard): this rank's exchange */
    uint64_t keys_sent;        /* phase-1 keys sent to other owners                        */
    uint64_t states_sent;      /* phase-2 accepted states shipped                          */
    uint64_t chunks;           /* exchange rounds (frontier chunks and drains of parked keys) */
    double exchange_seconds;   /* device time of the exchange rounds (exchange stream),    */
                               /* overlapped with the next round's expansion or not        */
    uint64_t stored_here;      /* distinct states this rank stores                         */
    /* RMC_FLAG_SPILL */
    uint64_t spilled;          /* states that left the device window (all spills of the run) */
    uint64_t spills;           /* spill events; with the links in HBM (a ring window whose  */
                               /* slots are reused, nothing copied) the passes of the ring  */
    double spill_seconds;      /* wall time of the spills (device-to-host + window shift;   */
                               /* 0 for the ring)                                           */
    /* sharded mode, continued */
    uint64_t parked;           /* keys parked because an owner's outbox was full; sent in   */
                               /* further rounds of the same level (never dropped)          */
    double exchange_wait_seconds; /* host wall time blocked on count read-backs and level ends */
    /* RMC_FLAG_SPILL, continued */
    int32_t spill_links_on_device; /* 1: the trace links (parent, lane) of spilled states stayed */
                                   /* in HBM and the window was a ring; 0: links on the host   */
    int32_t pad2;
    /* RMC_FLAG_VERIFY_STATES with RMC_FLAG_SPILL */
    uint64_t verified_spilled; /* hits (of `verified`) whose stored state had left the device */
                               /* window, compared with its host copy                       */
    uint64_t set_slots;        /* 8-B slots of the fingerprint set this run used (set_bytes) */
} rmc_result;

/* Per-level progress (TLC prints "Progress(D) ... states generated ..."). */
typedef struct rmc_level_stats {
    int32_t level;             /* level just completed (its successors were generated)  */
    int32_t pad;
    uint64_t generated;        /* cumulative generated                                  */
    uint64_t distinct;         /* cumulative distinct                                   */
    uint64_t new_states;       /* distinct states found at level+1                      */
    double seconds;            /* wall time since rmc_run_bfs started                   */
} rmc_level_stats;

/* Return non-zero to stop the search early. */
typedef int (*rmc_progress_fn)(const rmc_level_stats* stats, void* user);

/* A decoded state in neutral form, for traces and tests.  Field meanings are
 * the TLA+ variables of raft.tla:31-67; Nil = -1; roles 0/1/2 =
 * Follower/Candidate/Leader; mtype 0..3 = RequestVoteRequest,
 * RequestVoteResponse, AppendEntriesRequest, AppendEntriesResponse.
 * Fields that do not apply to a message type are 0. */
typedef struct rmc_entry { int32_t term, value; } rmc_entry;
typedef struct rmc_msg_view {
    int32_t mtype, mterm, msource, mdest;
    int32_t mlastLogTerm, mlastLogIndex;                      /* RequestVoteRequest    */
    int32_t mvoteGranted, mlog_len;                           /* RequestVoteResponse   */
    rmc_entry mlog[RMC_VIEW_LOG];
    int32_t mprevLogIndex, mprevLogTerm, mentries_len;        /* AppendEntriesRequest  */
    rmc_entry mentries[1];
    int32_t mcommitIndex;
    int32_t msuccess, mmatchIndex;                            /* AppendEntriesResponse */
    int32_t count;                                            /* bag multiplicity >= 1 */
} rmc_msg_view;
typedef struct rmc_state_view {
    int32_t n_servers, n_msgs;
    int32_t currentTerm[RMC_MAX_SERVERS];
    int32_t state[RMC_MAX_SERVERS];
    int32_t votedFor[RMC_MAX_SERVERS];
    int32_t commitIndex[RMC_MAX_SERVERS];
    int32_t log_len[RMC_MAX_SERVERS];
    rmc_entry log[RMC_MAX_SERVERS][RMC_VIEW_LOG];
    uint32_t votesResponded[RMC_MAX_SERVERS];   /* bitmask over server ids */
    uint32_t votesGranted[RMC_MAX_SERVERS];
    int32_t nextIndex[RMC_MAX_SERVERS][RMC_MAX_SERVERS];
    int32_t matchIndex[RMC_MAX_SERVERS][RMC_MAX_SERVERS];
    rmc_msg_view msgs[RMC_VIEW_MSGS];
} rmc_state_view;

/* One successor produced by rmc_expand (differential tests). */
typedef struct rmc_succ_view {
    uint64_t parent;           /* index into the input array                       */
    int32_t family;            /* 0..9 = Restart .. DropMessage (raft.tla:421-430)  */
    int32_t instance;          /* lane id within the state (DESIGN.md lane table)   */
    int32_t in_constraint;     /* 1 if the successor satisfies the CONSTRAINT       */
    int32_t pad;
    uint64_t fingerprint;
    rmc_state_view state;      /* valid when in_constraint                          */
} rmc_succ_view;

typedef struct rmc_ctx rmc_ctx;

/* ---- lifecycle ----------------------------------------------------------
 * rmc_create replaces TLC's model setup: cfg binding, ASSUME checks
 * (raft.tla:494-503, trivially true for model values), and FPSet/queue
 * allocation.  It validates the config and allocates the device state store,
 * fingerprint table and parent array on `cfg->device`. */
int rmc_create(const rmc_config* cfg, rmc_ctx** out);
void rmc_destroy(rmc_ctx* ctx);
const char* rmc_last_error(const rmc_ctx* ctx);   /* never NULL */
const char* rmc_version(void);                    /* "rmc <abi> gfx950 ..."           */

/* ---- breadth-first search ----------------------------------------------
 * Replaces TLC's BFS worker loop (ModelChecker: dequeue, getNextStates over
 * Next raft.tla:421-430, CONSTRAINT filter, FP64 + FPSet.put, invariant check,
 * enqueue).  Blocks until fixpoint, first violation, deadlock (when checked),
 * max_depth, or the callback asks to stop. */
int rmc_run_bfs(rmc_ctx* ctx, rmc_progress_fn cb, void* user);
/* Changes rmc_config.seed (fingerprint salt) for the next run on this ctx. */
int rmc_set_seed(rmc_ctx* ctx, uint64_t seed);
int rmc_get_result(const rmc_ctx* ctx, rmc_result* out);
/* Test hook of the verification mode: keep only the low `bits` fingerprint
 * bits (1..64), so collisions happen and must be reported.  Needs
 * RMC_FLAG_VERIFY_STATES. */
int rmc_set_fp_bits(rmc_ctx* ctx, int32_t bits);

/* Counterexample: the states from an initial state to the violating (or
 * deadlocked) state, in order, with the action family and lane of the step
 * into each state (-1 for the initial state).  Replaces TLC's trace
 * reconstruction from the states/ trace file ("State 1: ... State d").
 * *len receives the trace length even if it exceeds cap. */
int rmc_trace(rmc_ctx* ctx, rmc_state_view* states, int32_t* families, int32_t* instances,
              size_t cap, size_t* len);

/* ---- checkpoint / recovery (TLC -checkpoint / -recover) ----------------------
 * rmc_checkpoint: after rmc_run_bfs stopped at a level boundary (max_depth or
 * the progress callback), write the stored levels (states, parent refs, lanes),
 * the level table and the counters to `path`.  rmc_recover: on a ctx of the
 * same model (constants, bounds, flags, seed; capacity >= the checkpoint's
 * states), load them and rebuild the fingerprint set from the states; the next
 * rmc_run_bfs continues from the first unexpanded level, with cumulative
 * counts.  A sharded ctx (rmc_shard) writes and reads its own part,
 * <path>.rank<r>; every rank of the same world calls them, and the recovered
 * ctxs must be sharded the same way (rank, world) before rmc_recover. */
int rmc_checkpoint(rmc_ctx* ctx, const char* path);
int rmc_recover(rmc_ctx* ctx, const char* path);

/* ---- codec and successor enumeration (tests, Java driver printing) -------
 * rmc_state_bytes: bytes of one stored state for this config (packed, or the
 * wide layout's BFS record: 904 B compact or 5,080 B).
 * rmc_expand: run the SAME device successor code as the BFS on n caller
 * states (no dedup) and return every enabled lane's successor.  *n_out
 * receives the number of successors even if it exceeds cap. */
size_t rmc_state_bytes(const rmc_config* cfg);
int rmc_expand(rmc_ctx* ctx, const rmc_state_view* states, size_t n, rmc_succ_view* out,
               size_t cap, size_t* n_out);

/* ---- simulation (TLC -simulate; Smokeraft.cfg, config 4) ---------------------
 * Replaces TLC's Simulator: random behaviours, each from a random initial state
 * and then a uniformly random enabled successor per step, invariants checked on
 * every state.  smoke_k > 0 draws the initial states like SmokeInit
 * (Smokeraft.tla:64-76: one RandomSubset(k, .) per variable, k^9 states, over
 * SmokeNat = 0..smoke_nat, SmokeInt = -1..1, BoundedSeq(.,3)/(.,1) logs);
 * smoke_k = 0 starts from Init.  TLC's StopAfter (a 1-s budget,
 * Smokeraft.tla:88-92) is replaced by an explicit behaviour count.  Walks stay
 * within the config's bounds (max_term, max_log_len, max_msgs, max_dup: the
 * model's CONSTRAINT, or the packed capacity when it has none — the front-end
 * fills them in): RMC_SIM_WITHIN_CAPACITY draws each step uniformly among the
 * enabled successors within them (so behaviours run to `depth`);
 * RMC_SIM_TRUNCATE draws among all enabled successors and a draw beyond them
 * ends that behaviour (counted in `truncated`). */
#define RMC_SIM_WITHIN_CAPACITY 0
#define RMC_SIM_TRUNCATE 1
/* TLC's draw (its simulator's action choice, restated): Next's actions — each
 * instance of Restart .. AppendEntries (\E over the constant Server/Value sets
 * expands into one action each), Receive, DuplicateMessage and DropMessage
 * (\E m \in DOMAIN messages ranges over the state) one action each — are
 * visited from a uniformly random index with a random prime stride (primes
 * above the action count, so every action is visited); the first one with a
 * successor is taken and one of its successors drawn uniformly.  Not uniform
 * over the enabled actions: an action after a run of disabled ones is likelier.
 * Beyond the bounds it ends the behaviour like RMC_SIM_TRUNCATE.  Wide layout
 * only (rmc_simulate refuses it on the packed one). */
#define RMC_SIM_TLC 2
typedef struct rmc_sim_config {
    uint64_t behaviours;       /* random behaviours to run                        */
    int32_t depth;             /* states per behaviour (TLC -depth, default 100)  */
    int32_t smoke_k;           /* SmokeInit RandomSubset size k; 0 = Init         */
    int32_t smoke_nat;         /* SmokeNat = 0..smoke_nat (default 2)             */
    int32_t mode;              /* RMC_SIM_WITHIN_CAPACITY (0) or RMC_SIM_TRUNCATE */
    uint64_t seed;             /* RNG seed for the SmokeInit draws and the walks  */
} rmc_sim_config;
typedef struct rmc_sim_result {
    uint64_t behaviours, steps, init_states, truncated, deadlocked;
    int32_t violated_inv;      /* RMC_INV_* bit of the first violation, or 0      */
    int32_t violation_depth;   /* its state index in the behaviour (1 = initial)  */
    uint64_t violation_behaviour;
    double seconds;            /* wall time incl. the SmokeInit draw              */
    double kernel_seconds;     /* device time of the walks (HIP events)           */
} rmc_sim_result;
int rmc_simulate(rmc_ctx* ctx, const rmc_sim_config* sc, rmc_sim_result* out);
/* The initial states rmc_simulate draws for sc (SmokeInit, sc->smoke_k >= 1):
 * host-only, no device needed.  *n receives k^9 even if it exceeds cap. */
int rmc_smoke_init(const rmc_config* cfg, const rmc_sim_config* sc, rmc_state_view* states,
                   size_t cap, size_t* n);
/* Re-runs behaviour `behaviour` of the same rmc_sim_config and returns its states. */
int rmc_sim_replay(rmc_ctx* ctx, const rmc_sim_config* sc, uint64_t behaviour, rmc_state_view* states,
                   size_t cap, size_t* len);

/* ---- sharded BFS over several GPUs (one process or thread per GPU) ---------
 * Replaces TLC's distributed mode (TLCServer/TLCWorker with a partitioned
 * FPSet).  rmc_shard turns a ctx into rank `rank`
 * of `world`; rmc_run_bfs, rmc_get_result and rmc_trace then become
 * collectives that every rank calls, and return the GLOBAL result on every
 * rank.  A state is owned by the rank given by a hash of its servers 0 and 1
 * words (RMC_OWNER=2, default; 1: server 0 only; 0: by fingerprint, always
 * under SYMMETRY); each rank stores and expands the states it owns.
 * A level is expanded in rounds; each round's exchange is fingerprint-first
 * (two phases):
 *   1. a successor owned elsewhere (and not in this rank's lossy sent-cache)
 *      sends only its 8-byte key; the owner inserts the keys it receives
 *      into its fingerprint set and answers new / seen (1 byte per key);
 *   2. for the keys answered "new" the sender re-derives the successor and
 *      ships the state and its global parent ref ((rank << 48) | index, lane
 *      in bits 40-47); the owner stores it for the next level.
 * Rounds are pipelined: the next round's expansion runs while this round's
 * exchange is on the wire (two outbox sets, an exchange stream).  Per round
 * the host reads back two small count rows; one all-gather of the device
 * counters per level combines the level statistics.  A key whose owner's
 * outbox is full is parked and sent in a further round of the same level.
 * Replicated levels: a level of at most RMC_DIST_REP states (default 2^20) is
 * gathered whole on every rank (one all-gather of state records) and every
 * rank expands all of it, probing and storing only the successors it owns —
 * no key or state exchange for the small levels at either end of the search.
 * Deadlines: every collective and the communicator set-up run under
 * RMC_DIST_TIMEOUT_S (default 300 s; the RCCL communicator is non-blocking and
 * aborted on expiry, host-transport callbacks are expected to honour it too):
 * a stalled rank makes every other rank's rmc_run_bfs return RMC_E_HIP naming
 * the level, round and phase.
 * Transport: RCCL over xGMI (rccl_id = an id from rmc_rccl_unique_id on rank
 * 0, given to every rank; host = NULL), or a caller-supplied host transport
 * (rccl_id = NULL) whose callbacks move host buffers: alltoallv sends
 * send_bytes[d] bytes to rank d (blocks back to back in `send`) and receives
 * recv_bytes[s] from rank s (back to back in `recv`); allgather gathers
 * `bytes` from every rank into recv (rank order).  They return 0 on success.
 * keys_per_dest bounds the keys one round sends to one owner (0 = auto);
 * sent_cache_slots sizes the sent-cache (0 = auto).  Full-state verification
 * (RMC_FLAG_VERIFY_STATES) ships every remote successor and compares the ones
 * the owner had seen; checkpoints are per rank; RMC_FLAG_SPILL is single-GPU. */
typedef struct rmc_transport {
    void* user;
    int (*alltoallv)(void* user, const void* send, const uint64_t* send_bytes, void* recv,
                     const uint64_t* recv_bytes);
    int (*allgather)(void* user, const void* send, uint64_t bytes, void* recv);
} rmc_transport;
int rmc_rccl_unique_id(uint8_t id[128]);
int rmc_shard(rmc_ctx* ctx, int32_t rank, int32_t world, const uint8_t* rccl_id,
              const rmc_transport* host, uint64_t keys_per_dest, uint64_t sent_cache_slots);

/* ---- roofline microbenchmark -----------------------------------------------
 * Random 8-byte accesses into a table of table_bytes on `device`, 8 in flight
 * per thread, the access pattern of the fingerprint set: mode 0 = loads,
 * mode 1 = CAS.  *per_second receives accesses/s (device time, HIP events).
 * This is R_max of SURVEY.md §8d (no TLC analog). */
int rmc_probe_bench(int device, uint64_t table_bytes, uint64_t accesses, int mode, double* per_second);

/* ---- front-end -----------------------------------------------------------
 * Replaces TLC's SANY + cfg reading for this spec: reads a TLC model (root
 * .tla module, the modules it EXTENDS next to it, its .cfg, and raft.tla) and
 * fills *cfg — or refuses it, naming the construct the engine does not
 * compile.  The engine compiles lemmy/raft.tla:1-505 and nothing else, so:
 *  - raft.tla is read (raft_path, else $RMC_RAFT_TLA, else next to the
 *    model) and every top-level unit of its module body must match the
 *    compiled-in text (comments and whitespace normalised).  The one edit
 *    recognised is config 5's weakened quorum guard in BecomeLeader
 *    (raft.tla:197 `votesGranted[i] /= {}`), which sets RMC_FLAG_BUG_QUORUM.
 *    With no raft.tla on disk the call fails unless options has
 *    RMC_FRONT_BUILTIN_RAFT (then the compiled-in text is used, and said so);
 *  - CONSTANTS: model values, `X <- Def`, `Name = n`; Server and Value must
 *    be set literals of distinct model values;
 *  - CONSTRAINT(S): split into top-level conjuncts (bulleted or infix, through
 *    definition references); every conjunct must be one of
 *    `\A i \in Server : currentTerm[i] <= N /\ Len(log[i]) <= N`,
 *    `Cardinality(DOMAIN messages) <= N`, `\A m \in DOMAIN messages :
 *    messages[m] <= N` (<, =<, \leq too); anything else is refused;
 *  - INVARIANT(S): TypeOK, or a name from RMC_INV_* whose definition (with the
 *    model definitions it uses) is the compiled-in restatement;
 *  - `BecomeLeader <- Def`: Def must be the compiled-in bug variant;
 *  - SYMMETRY: exactly Permutations(Server) (or of Server's set definition);
 *  - simulation (RMC_FRONT_SIMULATE, TLC -simulate): `Init <- SmokeInit` must
 *    be Smokeraft's sampler (k and SmokeNat are read as its parameters); a
 *    CONSTRAINT that only reads TLCGet/TLCSet is a run budget, replaced by
 *    sim->behaviours; bounds the cfg does not give are the packed capacity.
 *  - an unconstrained field is refused unless options has
 *    RMC_FRONT_DEPTH_BOUNDED (see RMC_FLAG_UNBOUNDED_TERM).
 * On success `info` receives the provenance notes (which raft.tla was
 * verified, which overrides were recognised), on failure the error. */
#define RMC_FRONT_BUILTIN_RAFT (1u << 0)
#define RMC_FRONT_SIMULATE (1u << 1)
/* RMC_FRONT_DEPTH_BOUNDED: the caller bounds the depth (TLC -depth), so a model
 * whose CONSTRAINT leaves fields unbounded — or that has none, as MCraft.cfg
 * as shipped (MCraft.cfg:1-39) — is accepted with the RMC_FLAG_UNBOUNDED_*
 * bits set (rmc_create then requires max_depth > 0). */
#define RMC_FRONT_DEPTH_BOUNDED (1u << 2)
int rmc_model_from_files(const char* cfg_path, const char* tla_path, const char* raft_path,
                         uint32_t options, rmc_config* cfg, rmc_sim_config* sim,
                         char* info, size_t info_cap);
/* rmc_model_from_files for BFS / simulation models with raft_path = NULL and
 * RMC_FRONT_BUILTIN_RAFT taken from the environment (RMC_BUILTIN_RAFT=1).
 * `tla_path` may be NULL (the module next to cfg_path with the same stem). */
int rmc_config_from_files(const char* cfg_path, const char* tla_path, rmc_config* cfg,
                          char* err, size_t err_cap);
int rmc_sim_config_from_files(const char* cfg_path, const char* tla_path, rmc_config* cfg,
                              rmc_sim_config* sim, char* err, size_t err_cap);
/* TLC's location of an action of Next in raft.tla, as its counterexample
 * headers print it (`State k: <Action line L1, col C1 to line L2, col C2 of
 * module raft>`): the body of the action's definition.  `action` is a family
 * name of rmc.h's lane table, "UpdateTerm", or "Receive:<mtype>" for the
 * Receive disjunct of that message type (raft.tla:393-403).  out4 = L1, C1,
 * L2, C2. */
int rmc_action_location(const char* action, int32_t* out4);

#ifdef __cplusplus
}
#endif
#endif /* RMC_H_ */
