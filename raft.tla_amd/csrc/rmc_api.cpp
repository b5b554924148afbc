// rmc_api.cpp — the C ABI of librmc.so (include/rmc.h): context, BFS driver,
// codec, traces, and the differential-test entry point.
//
// Host side of the hot path: one HIP stream per context, one kernel launch
// (plus one 40-byte counter read-back) per BFS level.  The level loop
// replaces TLC's ModelChecker.runTLC / Worker loop.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>

#include "rmc_ctx.h"

using namespace rmc;

namespace {
const char* kVersion = "rmc 2 (raft.tla BFS, gfx950 HIP, packed-delta lanes, HBM fp set, RCCL sharding)";
}  // namespace

namespace rmc_host {

int fail(rmc_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}

int kcap_for(int max_msgs) { return max_msgs <= 4 ? 4 : 8; }

int validate(const rmc_config* c, std::string* why) {
    auto bad = [&](const char* s) { *why = s; return RMC_E_INVAL; };
    if (c->n_servers < 2 || c->n_servers > RMC_MAX_SERVERS) return bad("n_servers must be 2..5");
    if (c->n_values < 1 || c->n_values > RMC_MAX_VALUES) return bad("n_values must be 1..2");
    if (c->invariants & ~1023u) return bad("unknown invariant bit");
    if (c->flags & ~511u) return bad("unknown flag bit");
    if ((c->flags & RMC_UNBOUNDED_ANY) && c->max_depth <= 0)
        return bad("a model with unbounded fields (RMC_FLAG_UNBOUNDED_*) needs max_depth > 0 (TLC -depth)");
    if (wide_wanted(*c)) return validate_wide(c, why);  // bounds beyond the packed capacity
    if (c->max_term < 1 || c->max_term > RMC_MAX_TERM) return bad("max_term must be 1..14");
    if (c->max_log_len < 0 || c->max_log_len > RMC_MAX_LOG) return bad("max_log_len must be 0..3");
    if (c->max_msgs < 0 || c->max_msgs > RMC_MAX_MSGS) return bad("max_msgs must be 0..8");
    if (c->max_dup < 1 || c->max_dup > RMC_MAX_DUP) return bad("max_dup must be 1..3");
    return 0;
}

void fill_params(rmc_ctx* c) {
    const rmc_config& g = c->cfg;
    c->wide = wide_wanted(g) ? 1 : 0;
    if (c->wide) fill_wide_model(c);
    c->sh.S = g.n_servers;
    c->sh.K = kcap_for(g.max_msgs);
    c->sh.sym = (g.flags & RMC_FLAG_SYMMETRY) != 0;
    c->sh.verify = (g.flags & RMC_FLAG_VERIFY_STATES) != 0;
    c->NW = 2 * c->sh.S + c->sh.K;
    Params& P = c->P;
    P.V = g.n_values;
    P.max_term = g.max_term;
    P.max_log = g.max_log_len;
    P.max_msgs = g.max_msgs;
    P.max_dup = g.max_dup;
    P.bug_quorum = (g.flags & RMC_FLAG_BUG_QUORUM) ? 1 : 0;
    P.inv_mask = (int)g.invariants;
    P.symmetry = c->sh.sym ? 1 : 0;
    P.fp_mask = ~0ull;
    P.unbounded = (int)((g.flags >> 5) & 15u);  // RMC_FLAG_UNBOUNDED_TERM .. _DUP
    {  // commuting-diamond probe elimination (not under SYMMETRY; RMC_DIAMOND=0 turns it off)
        const char* e = getenv("RMC_DIAMOND");
        P.diamond = (!c->sh.sym && !(e && e[0] == '0')) ? 1 : 0;
    }
    const int S = c->sh.S, K = c->sh.K;
    const int sizes[10] = {S, S, S * S, S, S * VMAX, S, S * S, K, K, K};  // = Lanes<S,K>
    P.off[0] = 0;
    for (int f = 0; f < 10; ++f) P.off[f + 1] = P.off[f] + sizes[f];
    fill_lane_desc(P, S);
    // permutations of 0..S-1 in lexicographic order (identity first), 3 bits per id
    memset(&c->PT, 0, sizeof c->PT);
    {
        int a[5] = {0, 1, 2, 3, 4};
        int n = 0;
        do {
            u32 code = 0;
            for (int i = 0; i < S; ++i) code |= (u32)a[i] << (3 * i);
            c->PT.code[n] = code;
            ++n;
        } while (std::next_permutation(a, a + S));
        c->PT.np = n;
    }
}

int family_of(const Params& P, int lane) {
    if (lane == 255) return -1;
    for (int f = 0; f < 10; ++f)
        if (lane < P.off[f + 1]) return f;
    return -1;
}

// ---- codec ----------------------------------------------------------------------
int encode_view(const rmc_ctx* c, const rmc_state_view& v, u32* out, std::string* why) {
    const int S = c->sh.S, K = c->sh.K;
    const int VR = VR_SH, VG = VR_SH + S, NI = VR_SH + 2 * S, MI = VR_SH + 4 * S;
    auto bad = [&](const std::string& s) { *why = s; return RMC_E_INVAL; };
    if (v.n_servers != S) return bad("view n_servers differs from config");
    if (v.n_msgs < 0 || v.n_msgs > K) return bad("too many messages for the packed bag");
    for (int i = 0; i < S; ++i) {
        const int len = v.log_len[i];
        if (v.currentTerm[i] < 0 || v.currentTerm[i] > 15) return bad("currentTerm out of packed range");
        if (v.state[i] < 0 || v.state[i] > 2) return bad("state out of range");
        if (v.votedFor[i] < -1 || v.votedFor[i] >= S) return bad("votedFor out of range");
        if (v.commitIndex[i] < 0 || v.commitIndex[i] > 3) return bad("commitIndex out of packed range");
        if (len < 0 || len > LOG_CAP) return bad("log length out of packed range");
        u64 w = (u64)v.currentTerm[i] | ((u64)v.state[i] << ST_SH) |
                ((u64)(v.votedFor[i] < 0 ? NILV : (u32)v.votedFor[i]) << VF_SH) | ((u64)v.commitIndex[i] << CI_SH) |
                ((u64)len << LEN_SH);
        for (int x = 0; x < len; ++x) {
            const rmc_entry e = v.log[i][x];
            if (e.term < 0 || e.term > 15 || e.value < 0 || e.value > 1) return bad("log entry out of range");
            w |= (u64)(e.term | (e.value << 4)) << (LOG_SH + ENT_W * x);
        }
        if ((v.votesResponded[i] | v.votesGranted[i]) >> S) return bad("vote set out of range");
        w |= (u64)v.votesResponded[i] << VR;
        w |= (u64)v.votesGranted[i] << VG;
        for (int j = 0; j < S; ++j) {
            if (v.nextIndex[i][j] < 1 || v.nextIndex[i][j] > 4) return bad("nextIndex out of packed range");
            if (v.matchIndex[i][j] < 0 || v.matchIndex[i][j] > 3) return bad("matchIndex out of packed range");
            w |= (u64)(v.nextIndex[i][j] - 1) << (NI + 2 * j);
            w |= (u64)v.matchIndex[i][j] << (MI + 2 * j);
        }
        out[2 * i] = (u32)w;
        out[2 * i + 1] = (u32)(w >> 32);
    }
    std::vector<u32> slots;
    for (int q = 0; q < v.n_msgs; ++q) {
        const rmc_msg_view& m = v.msgs[q];
        if (m.mtype < 0 || m.mtype > 3) return bad("mtype out of range");
        if (m.msource < 0 || m.msource >= S || m.mdest < 0 || m.mdest >= S) return bad("message endpoint out of range");
        if (m.mterm < 0 || m.mterm > 15) return bad("mterm out of packed range");
        if (m.count < 1 || m.count > 3) return bad("message count out of packed range");
        u32 s = m_hdr((u32)m.mtype, (u32)m.msource, (u32)m.mdest, (u32)m.mterm);
        switch (m.mtype) {
            case RVQ:
                if (m.mlastLogTerm < 0 || m.mlastLogTerm > 15 || m.mlastLogIndex < 0 || m.mlastLogIndex > 3)
                    return bad("RequestVoteRequest field out of packed range");
                s |= ((u32)m.mlastLogTerm << 12) | ((u32)m.mlastLogIndex << 16);
                break;
            case RVP: {
                if (m.mlog_len < 0 || m.mlog_len > 3) return bad("mlog too long");
                u32 lg = (u32)m.mlog_len;
                for (int x = 0; x < m.mlog_len; ++x) {
                    if (m.mlog[x].term < 0 || m.mlog[x].term > 15 || m.mlog[x].value < 0 || m.mlog[x].value > 1)
                        return bad("mlog entry out of range");
                    lg |= (u32)(m.mlog[x].term | (m.mlog[x].value << 4)) << (2 + ENT_W * x);
                }
                s |= ((u32)(m.mvoteGranted != 0) << 12) | (lg << 13);
                break;
            }
            case AEQ: {
                if (m.mprevLogIndex < -1 || m.mprevLogIndex > 3 || m.mprevLogTerm < 0 || m.mprevLogTerm > 15 ||
                    m.mentries_len < 0 || m.mentries_len > 1 || m.mcommitIndex < 0 || m.mcommitIndex > 3)
                    return bad("AppendEntriesRequest field out of packed range");
                u32 e = 0;
                if (m.mentries_len) {
                    if (m.mentries[0].term < 0 || m.mentries[0].term > 15 || m.mentries[0].value < 0 ||
                        m.mentries[0].value > 1)
                        return bad("mentries entry out of range");
                    e = (u32)(m.mentries[0].term | (m.mentries[0].value << 4));
                }
                s |= ((u32)(m.mprevLogIndex + 1) << 12) | ((u32)m.mprevLogTerm << 15) |
                     ((u32)m.mentries_len << 19) | (e << 20) | ((u32)m.mcommitIndex << 25);
                break;
            }
            default:
                if (m.mmatchIndex < 0 || m.mmatchIndex > 3) return bad("mmatchIndex out of packed range");
                s |= ((u32)(m.msuccess != 0) << 12) | ((u32)m.mmatchIndex << 13);
        }
        for (u32 o : slots)
            if ((o & MSG_MASK) == s) return bad("duplicate message in bag view");
        slots.push_back(s | ((u32)m.count << 30));
    }
    std::sort(slots.begin(), slots.end(), [](u32 a, u32 b) { return a > b; });
    for (int q = 0; q < K; ++q) out[2 * S + q] = q < (int)slots.size() ? slots[q] : 0u;
    return 0;
}

void decode_state(const rmc_ctx* c, const u32* in, rmc_state_view* v) {
    const int S = c->sh.S, K = c->sh.K;
    const int VR = VR_SH, VG = VR_SH + S, NI = VR_SH + 2 * S, MI = VR_SH + 4 * S;
    memset(v, 0, sizeof *v);
    v->n_servers = S;
    for (int i = 0; i < S; ++i) {
        const u64 w = (u64)in[2 * i] | ((u64)in[2 * i + 1] << 32);
        v->currentTerm[i] = (int)w_ct(w);
        v->state[i] = (int)w_st(w);
        v->votedFor[i] = w_vf(w) == NILV ? -1 : (int)w_vf(w);
        v->commitIndex[i] = (int)w_ci(w);
        v->log_len[i] = (int)w_len(w);
        for (u32 x = 0; x < w_len(w); ++x) {
            v->log[i][x].term = (int)(w_ent(w, x) & 15u);
            v->log[i][x].value = (int)(w_ent(w, x) >> 4);
        }
        v->votesResponded[i] = bits(w, VR, S);
        v->votesGranted[i] = bits(w, VG, S);
        for (int j = 0; j < S; ++j) {
            v->nextIndex[i][j] = (int)bits(w, NI + 2 * j, 2) + 1;
            v->matchIndex[i][j] = (int)bits(w, MI + 2 * j, 2);
        }
    }
    int n = 0;
    for (int q = 0; q < K; ++q) {
        const u32 s = in[2 * S + q];
        if (!s) continue;
        rmc_msg_view& m = v->msgs[n++];
        m.mtype = (int)m_type(s);
        m.msource = (int)m_src(s);
        m.mdest = (int)m_dst(s);
        m.mterm = (int)m_term(s);
        m.count = (int)m_cnt(s);
        switch (m.mtype) {
            case RVQ:
                m.mlastLogTerm = (int)((s >> 12) & 15u);
                m.mlastLogIndex = (int)((s >> 16) & 3u);
                break;
            case RVP: {
                m.mvoteGranted = (int)((s >> 12) & 1u);
                const u32 lg = (s >> 13) & 0x1FFFFu;
                m.mlog_len = (int)(lg & 3u);
                for (int x = 0; x < m.mlog_len; ++x) {
                    const u32 e = (lg >> (2 + ENT_W * x)) & 31u;
                    m.mlog[x].term = (int)(e & 15u);
                    m.mlog[x].value = (int)(e >> 4);
                }
                break;
            }
            case AEQ: {
                m.mprevLogIndex = (int)((s >> 12) & 7u) - 1;
                m.mprevLogTerm = (int)((s >> 15) & 15u);
                m.mentries_len = (int)((s >> 19) & 1u);
                const u32 e = (s >> 20) & 31u;
                if (m.mentries_len) {
                    m.mentries[0].term = (int)(e & 15u);
                    m.mentries[0].value = (int)(e >> 4);
                }
                m.mcommitIndex = (int)((s >> 25) & 3u);
                break;
            }
            default:
                m.msuccess = (int)((s >> 12) & 1u);
                m.mmatchIndex = (int)((s >> 13) & 3u);
        }
    }
    v->n_msgs = n;
}

void init_view(const rmc_config& g, rmc_state_view* v) {  // Init raft.tla:113-129
    memset(v, 0, sizeof *v);
    v->n_servers = g.n_servers;
    for (int i = 0; i < g.n_servers; ++i) {
        v->currentTerm[i] = 1;
        v->state[i] = 0;
        v->votedFor[i] = -1;
        for (int j = 0; j < g.n_servers; ++j) v->nextIndex[i][j] = 1;
    }
}

int reset_counters(rmc_ctx* c, bool keep_count) {
    Counters h{};
    h.count = keep_count ? c->h_ctr->count : 0;
    h.viol = ~0ull;
    h.deadlock = ~0ull;
    *c->h_ctr = h;
    HIPCHK(c, hipMemcpyAsync(c->B.ctr, c->h_ctr, sizeof(Counters), hipMemcpyHostToDevice, c->st));
    return 0;
}

// The checkpoint file of this ctx's part: <path> on one GPU, <path>.rank<r>
// for rank r of a sharded search.
std::string shard_path(const rmc_ctx* c, const char* path) {
    if (!c->dist.on || c->dist.world <= 1) return path;
    return std::string(path) + ".rank" + std::to_string(c->dist.rank);
}

std::string capacity_message(const rmc_ctx* c, u32 overflow, int depth) {
    const u32 f = (overflow >> 8) & 15u;
    if (!f) return "";
    std::string what;
    if (f & 1) what += std::string(what.empty() ? "" : ", ") + "currentTerm > " + std::to_string(c->cfg.max_term);
    if (f & 2) what += std::string(what.empty() ? "" : ", ") + "Len(log) > " + std::to_string(c->cfg.max_log_len);
    if (f & 4) what += std::string(what.empty() ? "" : ", ") + "Cardinality(DOMAIN messages) > " +
                       std::to_string(c->cfg.max_msgs);
    if (f & 8) what += std::string(what.empty() ? "" : ", ") + "messages[m] > " + std::to_string(c->cfg.max_dup);
    return "a successor of a level-" + std::to_string(depth) + " state needs " + what + ": beyond the " +
           (c->wide ? "wide" : "packed") +
           " layout's capacity of a field no CONSTRAINT bounds (lower the depth bound or add a CONSTRAINT)";
}

int read_counters(rmc_ctx* c) {
    HIPCHK(c, hipMemcpyAsync(c->h_ctr, c->B.ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return 0;
}

// ---- frontier spill (RMC_FLAG_SPILL) ---------------------------------------------
// TLC keeps its state queue in the states/ directory and a trace file of
// (parent, action) records from which it re-derives counterexample states
// (SURVEY.md §8f rank 4).  Here the fingerprint set and the state window stay
// in HBM; spilled states keep only their trace links in host memory.  Kernels
// index states by their global index through device pointers biased by -base.
void spill_rebase(rmc_ctx* c, u64 base) {
    SpillState& X = c->spill;
    X.base = base;
    if (X.dev_links) {  // the ring window (DevBufs.wmask): nothing moves, base = the oldest resident state
        c->B.store = X.store;
        c->B.parent = X.parent;
        c->B.act = X.act;
        c->B.foot = X.foot;
        c->B.cls = X.cls;
        c->B.cap = X.total_cap;
        return;
    }
    const uintptr_t nw = (uintptr_t)c->NW;
    c->B.store = (u32*)((uintptr_t)X.store - (uintptr_t)base * nw * 4);
    const u64 lb = X.dev_links ? 0 : base;  // device links: indexed by global index, never rebased
    c->B.parent = (u64*)((uintptr_t)X.parent - (uintptr_t)lb * 8);
    c->B.act = (uint8_t*)((uintptr_t)X.act - (uintptr_t)lb);
    c->B.foot = (u64*)((uintptr_t)X.foot - (uintptr_t)base * 8);
    c->B.cls = (uint8_t*)((uintptr_t)X.cls - (uintptr_t)base);
    // device links hold total_cap states: no store index may pass it
    c->B.cap = X.dev_links ? std::min(base + X.win, X.total_cap) : base + X.win;
}

// Address space for the trace links of every state the set can hold; pages
// are only backed once a spill touches them.
int spill_reserve(rmc_ctx* c) {
    SpillState& X = c->spill;
    X.h_bytes = (size_t)X.total_cap * 9;
    void* m = mmap(nullptr, X.h_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) {
        X.h_bytes = 0;
        return fail(c, RMC_E_NOMEM, "spill: cannot reserve host address space for the trace links");
    }
    (void)madvise(m, X.h_bytes, MADV_HUGEPAGE);  // 2 MiB faults: fewer, cheaper first touches
    X.h_parent = (u64*)m;
    X.h_act = (uint8_t*)m + (size_t)X.total_cap * 8;
    X.faulted = 0;
    return 0;
}

void spill_free(rmc_ctx* c) {
    if (c->spill.ahead.joinable()) c->spill.ahead.join();
    if (c->spill.h_bytes) munmap(c->spill.h_parent, c->spill.h_bytes);
    c->spill.h_parent = nullptr;
    c->spill.h_act = nullptr;
    c->spill.h_bytes = 0;
}

// Touch fresh host pages from several threads: a device-to-host copy into
// untouched pageable memory runs at page-fault speed (~13 GB/s measured),
// into touched memory at ~48 GB/s (profiles/r02/host_link_rates.jsonl).
static void prefault(void* p, size_t n) {
    const int T = (int)std::min<size_t>(8, std::max<size_t>(1, n >> 26));
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([=] {  // one store per 4 KiB page backs it (fresh pages read as zero)
            volatile char* q = (volatile char*)p;
            for (size_t o = n * t / T, hi = n * (t + 1) / T; o < hi; o += 4096) q[o] = 0;
        });
    for (auto& x : th) x.join();
}

// Move the trace links of the device-resident states [base, a) to the host
// and shift [a, count) to the start of the window.  (With the links in HBM the
// window is a ring and nothing ever moves: see the launch loop.)
int spill_to(rmc_ctx* c, u64 a, u64 count) {
    SpillState& X = c->spill;
    const u64 n = a - X.base;
    if (!n) return 0;
    const auto t0 = std::chrono::steady_clock::now();
    const u64 W = (u64)c->NW * 4;
    u64* hp = X.h_parent + X.base;
    uint8_t* ha = X.h_act + X.base;
    if (X.ahead.joinable()) X.ahead.join();
    if (a > X.faulted) {  // what the background touch did not reach
        const u64 f0 = std::max(X.faulted, X.base);
        prefault(X.h_parent + f0, (a - f0) * 8);
        prefault(X.h_act + f0, a - f0);
        X.faulted = a;
    }
    HIPCHK(c, hipMemcpyAsync(hp, X.parent, n * 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipMemcpyAsync(ha, X.act, n, hipMemcpyDeviceToHost, c->st));
    if (X.h_state) {  // verification: the states too (the window's first n are [base, a))
        HIPCHK(c, hipMemcpyAsync(X.h_state + X.base * (u64)c->NW, X.store, n * W, hipMemcpyDeviceToHost, c->st));
        X.hcopied = a;
    }
    // shift in pieces of at most n states: no piece overlaps its own destination,
    // and stream order keeps every source read before a later piece overwrites it
    const u64 m = count - a;
    for (u64 off = 0; off < m; off += n) {
        const u64 k = std::min(n, m - off);
        HIPCHK(c, hipMemcpyAsync((char*)X.store + off * W, (char*)X.store + (n + off) * W, k * W,
                                 hipMemcpyDeviceToDevice, c->st));
        HIPCHK(c, hipMemcpyAsync(X.parent + off, X.parent + n + off, k * 8, hipMemcpyDeviceToDevice, c->st));
        HIPCHK(c, hipMemcpyAsync(X.act + off, X.act + n + off, k, hipMemcpyDeviceToDevice, c->st));
        HIPCHK(c, hipMemcpyAsync(X.foot + off, X.foot + n + off, k * 8, hipMemcpyDeviceToDevice, c->st));
        HIPCHK(c, hipMemcpyAsync(X.cls + off, X.cls + n + off, k, hipMemcpyDeviceToDevice, c->st));
    }
    HIPCHK(c, hipStreamSynchronize(c->st));
    spill_rebase(c, a);
    // the next spill takes at most a window's worth: back those pages while the
    // device expands
    const u64 f1 = std::min(X.total_cap, a + X.win);
    if (f1 > X.faulted) {
        const u64 f0 = X.faulted;
        X.faulted = f1;
        X.ahead = std::thread([&X, f0, f1] {
            prefault(X.h_parent + f0, (f1 - f0) * 8);
            prefault(X.h_act + f0, f1 - f0);
        });
    }
    c->res.spilled += n;
    c->res.spills += 1;
    c->res.spill_seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

// ---- verification + spill --------------------------------------------------------
// Full-state verification compares every fingerprint hit with the stored state
// that owns the slot.  A spilled search overwrites (ring) or drops (shifted
// window) the device copies of old states, so each state is copied to a host
// mirror before its device copy goes, and a hit on such an owner is parked by
// the expansion kernel (B.hbuf) and compared after the launch with the owner's
// host copy (k_verify_host).  Most duplicates are of recent states, so few hits
// take that path.
int verify_spill_reserve(rmc_ctx* c) {
    SpillState& X = c->spill;
    X.hs_bytes = (size_t)X.total_cap * (size_t)c->NW * 4;
    void* m = mmap(nullptr, X.hs_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) {
        X.hs_bytes = 0;
        return fail(c, RMC_E_NOMEM, "verification + spill: cannot reserve host address space for the states");
    }
    (void)madvise(m, X.hs_bytes, MADV_HUGEPAGE);
    X.h_state = (u32*)m;
    X.ostage_cap = 1ull << 22;
    c->B.hcap = 1ull << 26;
    if (hipHostMalloc(&X.h_ostage, X.ostage_cap * (u64)c->NW * 4, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&X.d_ostage, X.ostage_cap * (u64)c->NW * 4) != hipSuccess ||
        hipMalloc(&c->B.hbuf, c->B.hcap * 16) != hipSuccess)
        return fail(c, RMC_E_NOMEM, "verification + spill: staging allocation failed");
    return 0;
}

// Ring window: copy the states [hcopied, upto) — all below the launch's frontier,
// so final, and not yet overwritten — to the host mirror (up to two pieces).
int verify_copy_out(rmc_ctx* c, u64 upto) {
    SpillState& X = c->spill;
    const u64 W = (u64)c->NW * 4;
    while (X.hcopied < upto) {
        const u64 i = X.hcopied, sl = i & c->B.wmask;
        const u64 n = std::min(upto - i, X.win - sl);
        HIPCHK(c, hipMemcpyAsync((char*)X.h_state + i * W, (char*)X.store + sl * W, n * W, hipMemcpyDeviceToHost,
                                 c->st));
        X.hcopied = i + n;
    }
    return 0;
}

// The n hits the last launch parked in B.hbuf {parent, owner index | lane << 56}:
// stage the owners' host copies (batches of ostage_cap) and compare on the device.
int verify_host_hits(rmc_ctx* c, u64 n) {
    SpillState& X = c->spill;
    if (n > c->B.hcap) return fail(c, RMC_E_CAPACITY, "verification buffer full");
    std::vector<u64> rec(2 * n);
    HIPCHK(c, hipMemcpyAsync(rec.data(), c->B.hbuf, n * 16, hipMemcpyDeviceToHost, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    const u64 NW = (u64)c->NW;
    for (u64 off = 0; off < n; off += X.ostage_cap) {
        const u64 m = std::min(X.ostage_cap, n - off);
        for (u64 q = 0; q < m; ++q) {
            const u64 ix = rec[2 * (off + q) + 1] & ((1ull << 56) - 1);
            if (ix >= X.hcopied)
                return fail(c, RMC_E_HIP, "verification: a spilled owner (index " + std::to_string(ix) +
                                              ") has no host copy");
            memcpy(X.h_ostage + q * NW, X.h_state + ix * NW, NW * 4);
        }
        HIPCHK(c, hipMemcpyAsync(X.d_ostage, X.h_ostage, m * NW * 4, hipMemcpyHostToDevice, c->st));
        HIPCHK(c, launch(c->sh, 15, c->P, c->PT, c->B, m, off, X.d_ostage, nullptr, 0, nullptr, c->st));
        HIPCHK(c, hipStreamSynchronize(c->st));  // the pinned stage is refilled next
    }
    HIPCHK(c, hipMemsetAsync(&c->B.ctr->hcount, 0, 8, c->st));
    c->h_ctr->hcount = 0;
    X.host_hits += n;
    return 0;
}

// The trace link (parent index, action lane) of any stored state.
int read_link(rmc_ctx* c, u64 idx, u64* parent, uint8_t* act) {
    if (c->spill.on && !c->spill.dev_links && idx < c->spill.base) {
        *parent = c->spill.h_parent[idx];
        *act = c->spill.h_act[idx];
        return 0;
    }
    HIPCHK(c, hipMemcpy(parent, c->B.parent + idx, 8, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(act, c->B.act + idx, 1, hipMemcpyDeviceToHost));
    return 0;
}

}  // namespace rmc_host

using namespace rmc_host;

extern "C" {

const char* rmc_version(void) { return kVersion; }

const char* rmc_last_error(const rmc_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

size_t rmc_state_bytes(const rmc_config* cfg) {
    if (!cfg) return 0;
    if (wide_wanted(*cfg)) return wide_record_bytes(*cfg);
    return (size_t)(2 * cfg->n_servers + kcap_for(cfg->max_msgs)) * 4u;
}

int rmc_create(const rmc_config* cfg, rmc_ctx** out) {
    if (!cfg || !out) return RMC_E_INVAL;
    *out = nullptr;
    std::string why;
    if (int rc = validate(cfg, &why)) {
        fprintf(stderr, "rmc_create: %s\n", why.c_str());
        return rc;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg->device || cfg->device < 0) {
        fprintf(stderr, "rmc_create: no HIP device %d\n", cfg->device);
        return RMC_E_NOGPU;
    }
    rmc_ctx* c = new rmc_ctx();
    c->cfg = *cfg;
    fill_params(c);
    auto bail = [&](int rc) {
        fprintf(stderr, "rmc_create: %s\n", c->err.c_str());
        rmc_destroy(c);
        return rc;
    };
    if (hipSetDevice(cfg->device) != hipSuccess) { c->err = "hipSetDevice failed"; return bail(RMC_E_NOGPU); }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) { c->err = "hipGetDeviceProperties failed"; return bail(RMC_E_NOGPU); }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        c->err = std::string("device is ") + prop.gcnArchName + ", librmc is built for gfx950 only";
        return bail(RMC_E_NOGPU);
    }
    if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        c->err = "stream/event creation failed";
        return bail(RMC_E_HIP);
    }
    if (hipHostMalloc(&c->h_ctr, sizeof(Counters), hipHostMallocDefault) != hipSuccess) {
        c->err = "pinned allocation failed";
        return bail(RMC_E_NOMEM);
    }
    memset(c->h_ctr, 0, sizeof(Counters));
    if (c->wide) {  // bounds beyond the packed capacity: the wide layout (rmc_wide.cpp)
        if (int rc = create_wide(c)) return bail(rc);
        *out = c;
        return 0;
    }

    // ---- capacity: state store + parents + lanes + fingerprint set (load <= 0.5)
    const u64 per_state = (u64)c->NW * 4 + 8 + 1 + 8 + 1;  // state, parent, lane, footprint, class
    const bool spill = (cfg->flags & RMC_FLAG_SPILL) != 0;
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    const u64 budget = (u64)((double)fr * 0.80);
    u64 cap = cfg->state_capacity;
    // rmc_config.set_bytes (TLC -fpmem): the set's slots, the largest power of two that fits
    u64 set_slots = set_slots_of(cfg->set_bytes);
    if (set_slots && cap) {
        // set_bytes is an upper bound: halved (down to load 1/2) until the store fits
        // beside it — the states, or spilling the device trace links and the window
        // the spill sizing below asks for (need_win)
        const u64 sb = c->sh.verify ? 16 : 8;
        const u64 need_win = cfg->device_window ? cfg->device_window : cap / (c->sh.verify ? 8 : 4);
        const u64 store = spill ? cap * 9 + need_win * (per_state - 9) : cap * per_state;
        while (set_slots > 1024 && set_slots / 2 >= 2 * cap && set_slots * sb + store > budget) set_slots >>= 1;
    }
    if (set_slots && cap > set_slots / 2) {
        c->err = "state_capacity " + std::to_string(cap) + " exceeds what a set of set_bytes " +
                 std::to_string(cfg->set_bytes) + " holds (" + std::to_string(set_slots / 2) + " states)";
        return bail(RMC_E_INVAL);
    }
    if (cap == 0 && set_slots) {
        // the given set holds set_slots / 2 states; the store fills what the set leaves
        const u64 fixed = set_slots * (c->sh.verify ? 16 : 8);
        cap = set_slots / 2;
        if (!spill) cap = std::min<u64>(cap, (budget - std::min<u64>(budget, fixed)) / per_state);
    } else if (cap == 0) {
        // table <= 4 slots per state after pow2 rounding (+ as many sidx words when verifying);
        // spilling: the largest set of at most half the budget, two slots per state
        if (spill && c->sh.verify) {  // the set and its slot -> index map: 16 B per slot, <= 2/3 of the budget
            u64 sl = 1ull << 20;
            while (sl * 32 <= budget / 3 * 2) sl <<= 1;
            cap = sl / 2;
        } else if (spill) {
            u64 sl = 1ull << 20;
            while (sl * 16 <= budget / 2) sl <<= 1;  // 8 B * (2 sl) <= budget / 2
            cap = sl / 2;
        } else {
            cap = budget / (per_state + (c->sh.verify ? 64 : 32));
        }
        cap = std::min<u64>(cap, 1ull << 36);
    }
    cap = std::max<u64>(cap, 1024);
    u64 slots = 1;
    while (slots < 2 * cap) slots <<= 1;
    if (set_slots) slots = std::max(slots, set_slots);
    c->table_slots = slots;
    u64 win = cap;  // states resident on the device
    // spilling: the trace links of every state stay on the device (9 B each) when
    // that leaves a window of at least a quarter of the states; otherwise, or with
    // RMC_SPILL_HOST_LINKS=1, they move to the host with the spilled levels
    bool dev_links = false;
    u64 link_cap = win;
    if (spill) {
        // (verification: the slot -> index map and the two hit buffers, 1 GB each)
        const u64 fixed = slots * (c->sh.verify ? 16 : 8) + (c->sh.verify ? (2ull << 30) : 0);
        const u64 rest = budget - std::min<u64>(budget, fixed);
        const char* hl = getenv("RMC_SPILL_HOST_LINKS");
        const u64 wbytes = per_state - 9;  // state, footprint, class
        // verification keeps a smaller ring (its set is twice the size): an eighth of the states
        const u64 need_win = cfg->device_window ? cfg->device_window : cap / (c->sh.verify ? 8 : 4);
        dev_links = !(hl && atoi(hl)) && rest > cap * 9 && (rest - cap * 9) / wbytes >= need_win;
        win = cfg->device_window;
        if (win == 0) win = dev_links ? (rest - cap * 9) / wbytes : rest / per_state;
        win = std::max<u64>(std::min<u64>(win, cap), 1024);
        if (dev_links) {
            // the window is a ring of a power of two states (DevBufs.wmask): a
            // given window rounds up, librmc's own sizing down
            u64 p2 = 1024;
            while (p2 < win) p2 <<= 1;
            win = (cfg->device_window || p2 == win) ? p2 : p2 >> 1;
        }
        link_cap = dev_links ? cap : win;
    }
    c->B.cap = win;
    c->B.tmask = slots - 1;
    c->B.wmask = dev_links ? win - 1 : ~0ull;
    if (hipMalloc(&c->B.store, win * (u64)c->NW * 4) != hipSuccess ||
        hipMalloc(&c->B.parent, link_cap * 8) != hipSuccess || hipMalloc(&c->B.act, link_cap) != hipSuccess ||
        hipMalloc(&c->B.foot, win * 8) != hipSuccess || hipMalloc(&c->B.cls, win) != hipSuccess ||
        hipMalloc(&c->B.table, slots * 8) != hipSuccess || hipMalloc(&c->B.ctr, sizeof(Counters)) != hipSuccess ||
        hipMalloc(&c->B.word, (1ull << kMaxLaunchLog2) * 2) != hipSuccess ||  // presorted windows of one launch
        hipMalloc(&c->d_staged, (size_t)c->NW * 4 * 64) != hipSuccess) {
        c->err = "device allocation failed (capacity " + std::to_string(win) + " states)";
        return bail(RMC_E_NOMEM);
    }
    c->spill.on = spill ? 1 : 0;
    c->spill.dev_links = dev_links ? 1 : 0;
    c->spill.win = win;
    c->spill.total_cap = cap;
    c->spill.store = c->B.store;
    c->spill.parent = c->B.parent;
    c->spill.act = c->B.act;
    c->spill.foot = c->B.foot;
    c->spill.cls = c->B.cls;
    // classes are a layout hint (any value is a valid class): zero them once so
    // recovered or never-written states sort deterministically
    if (hipMemset(c->B.cls, 0, win) != hipSuccess) {
        c->err = "hipMemset failed";
        return bail(RMC_E_HIP);
    }
    if (spill && !dev_links && spill_reserve(c)) return bail(RMC_E_NOMEM);
    if (c->sh.sym) {  // successors with tied signatures, canonicalised by k_ties after each launch
        // a lane defers at most one tied successor, so launches of at most
        // tie_cap / lanes states cannot overflow it (run_bfs sizes them so):
        // room for full 2^24-state launches (6.4 GB for S = 3, K = 4; smaller
        // launches cost ~6 % on the MCraftBench bounds), halved until it fits
        c->B.tie_cap = (u64)c->P.off[10] << 24;
        while (hipMalloc(&c->B.ties, c->B.tie_cap * 8) != hipSuccess) {
            c->B.ties = nullptr;
            c->B.tie_cap >>= 1;
            if (c->B.tie_cap < (1ull << 20)) break;
        }
        if (!c->B.ties) {
            c->err = "device allocation failed (symmetry tie buffer)";
            return bail(RMC_E_NOMEM);
        }
    }
    if (c->sh.verify) {  // slot -> store index (8 B per slot) + deferred-hit buffer (16 B per record)
        c->B.vcap = 1ull << 26;
        if (hipMalloc(&c->B.sidx, slots * 8) != hipSuccess || hipMalloc(&c->B.vbuf, c->B.vcap * 16) != hipSuccess) {
            c->err = "device allocation failed (verification buffers)";
            return bail(RMC_E_NOMEM);
        }
        if (spill && verify_spill_reserve(c)) return bail(RMC_E_NOMEM);
    }
    c->B.rank = 0;
    c->B.world = 1;
    c->B.ref_tag = 0;
    *out = c;
    return 0;
}

void rmc_destroy(rmc_ctx* c) {
    if (!c) return;
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->wide) destroy_wide(c);
    spill_free(c);
    // the unbiased allocations (B.* may be rebased by a spill)
    (void)hipFree(c->spill.store ? c->spill.store : c->B.store);
    (void)hipFree(c->spill.parent ? c->spill.parent : c->B.parent);
    (void)hipFree(c->spill.act ? c->spill.act : c->B.act);
    (void)hipFree(c->spill.foot ? c->spill.foot : c->B.foot);
    (void)hipFree(c->spill.cls ? c->spill.cls : c->B.cls);
    (void)hipFree(c->B.table);
    (void)hipFree(c->B.ctr);
    (void)hipFree(c->B.word);
    (void)hipFree(c->d_staged);
    free_dist(c);
    (void)hipFree(c->B.sidx);
    (void)hipFree(c->B.vbuf);
    (void)hipFree(c->B.hbuf);
    (void)hipFree(c->spill.d_ostage);
    if (c->spill.h_ostage) (void)hipHostFree(c->spill.h_ostage);
    if (c->spill.hs_bytes) munmap(c->spill.h_state, c->spill.hs_bytes);
    (void)hipFree(c->B.ties);
    if (c->h_ctr) (void)hipHostFree(c->h_ctr);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

// The most new states one state's expansion can yield: every lane yields at most
// one, and the guards of raft.tla's Next (raft.tla:421-430) enable per server i at
// most Restart + Timeout (a Follower, :136,146), Restart + Timeout + S x RequestVote +
// BecomeLeader (a Candidate, :157-158,195-196) or Restart + V x ClientRequest +
// AdvanceCommitIndex + (S - 1) x AppendEntries (a Leader, :171-173,206-207,219-220),
// plus Receive, Duplicate and Drop per bag slot.  The spill window sizes its
// launches by this bound (RMC_LANE_BOUND=0: every lane, the round-5 bound).
static u64 max_new_per_state(const rmc_ctx* c) {
    const u64 lanes = (u64)c->P.off[10];
    static const bool all_lanes = [] {
        const char* e = getenv("RMC_LANE_BOUND");
        return e && atoi(e) == 0;
    }();
    if (all_lanes) return lanes;
    const u64 S = (u64)c->sh.S, V = (u64)c->P.V, K = (u64)(c->P.off[8] - c->P.off[7]);
    const u64 per_server = std::max<u64>(std::max<u64>(2, S + 3), S + V + 1);
    return std::min<u64>(lanes, S * per_server + 3 * K);
}

int rmc_run_bfs(rmc_ctx* c, rmc_progress_fn cb, void* user) {
    if (!c) return RMC_E_INVAL;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (c->wide) return run_bfs_wide(c, cb, user);
    if (c->dist.on) return run_bfs_sharded(c, cb, user);
    const auto t0 = std::chrono::steady_clock::now();
    auto secs = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    const bool resume = c->resume != 0;  // rmc_recover restored store, set and counters
    c->resume = 0;
    c->have_target = 0;
    int depth = 0;
    if (resume) {
        c->res.left_on_queue = 0;
        c->res.seconds = 0;
        HIPCHK(c, set_fp_salt(c->sh, c->cfg.seed, c->set_epoch, c->st));
        c->h_ctr->count = c->level_start.back();
        if (int rc = reset_counters(c, true)) return rc;
        depth = c->resume_depth;
    } else {
    c->res = rmc_result{};
    c->res.set_slots = c->table_slots;
    c->res.spill_links_on_device = c->spill.on && c->spill.dev_links;
    c->walked = 0;
    c->level_start.clear();
    if (c->spill.on) {
        spill_rebase(c, 0);
        SpillState& X = c->spill;
        const u64 f1 = std::min(X.total_cap, X.win);  // back the first spill's pages meanwhile
        if (!X.dev_links && !X.ahead.joinable() && f1 > X.faulted) {
            const u64 f0 = X.faulted;
            X.faulted = f1;
            X.ahead = std::thread([&X, f0, f1] {
                prefault(X.h_parent + f0, (f1 - f0) * 8);
                prefault(X.h_act + f0, f1 - f0);
            });
        }
    }
    // The set epoch (raft_packed.h c_set_ep): a run on a ctx whose set holds the
    // tagged entries of an earlier run takes the next epoch and clears nothing —
    // their slots read as empty.  The first run of a ctx, every 255th and runs
    // with verification (whose slot -> state map is cleared anyway) clear the set
    // (RMC_SET_EPOCH=0: every run clears; =N: at most N epochs between clears).
    const char* epe = getenv("RMC_SET_EPOCH");  // (read per run: tests vary it)
    const u32 ep_max = epe ? (u32)std::min(255, std::max(0, atoi(epe))) : 255u;
    const bool tagged = ep_max > 0 && !c->sh.verify;
    if (tagged && c->set_epoch >= 1 && c->set_epoch < ep_max) {
        c->set_epoch += 1;
    } else {
        HIPCHK(c, launch_fill(c->B.table, c->table_slots * 8, 0, c->st));
        c->set_epoch = tagged ? 1 : 0;
    }
    if (c->sh.verify) HIPCHK(c, launch_fill(c->B.sidx, c->table_slots * 8, 0xFF, c->st));
    HIPCHK(c, set_fp_salt(c->sh, c->cfg.seed, c->set_epoch, c->st));
    if (int rc = reset_counters(c, false)) return rc;
    c->B.vlo = 0;
    c->spill.hcopied = 0;
    c->spill.host_hits = 0;

    // ---- Init (raft.tla:125-129): one initial state
    rmc_state_view iv;
    init_view(c->cfg, &iv);
    std::vector<u32> packed((size_t)c->NW);
    std::string why;
    if (encode_view(c, iv, packed.data(), &why)) return fail(c, RMC_E_INVAL, why);
    HIPCHK(c, hipMemcpyAsync(c->d_staged, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, launch(c->sh, 1, c->P, c->PT, c->B, 1, 0, c->d_staged, nullptr, 0, nullptr, c->st));
    if (int rc = read_counters(c)) return rc;
    c->res.generated = 1;
    c->level_start.push_back(0);
    c->level_start.push_back(c->h_ctr->count);
    if (c->sh.verify)
        HIPCHK(c, launch(c->sh, 5, c->P, c->PT, c->B, 0, c->h_ctr->count, nullptr, nullptr, 0, nullptr, c->st));
    depth = c->h_ctr->count ? 1 : 0;
    if (c->h_ctr->viol != ~0ull) {
        c->res.violated_inv = 1 << (int)(c->h_ctr->viol & 15);
        c->res.violation_depth = 1;
        c->have_target = 1;
        c->target_idx = c->h_ctr->viol >> 4;
    }
    }  // !resume
    // states per expansion launch: at most kMaxLaunch (B.word holds one launch's
    // presorted positions), and a level is cut into EQUAL launches, so no launch
    // is a small remainder that leaves most of the resident grid idle
    // (RMC_LAUNCH_LOG2: a smaller cap, A/B)
    static const u64 CHUNK = [] {
        const char* e = getenv("RMC_LAUNCH_LOG2");
        const int l = e ? std::max(16, std::min(kMaxLaunchLog2, atoi(e))) : kMaxLaunchLog2;
        return 1ull << l;
    }();
    while (!c->have_target) {
        const u64 lo = c->level_start[depth - 1], hi = c->level_start[depth];
        if (lo == hi) break;  // fixpoint
        if (c->cfg.max_depth > 0 && depth >= c->cfg.max_depth) {
            c->res.left_on_queue = hi - lo;
            break;
        }
        if (int rc = reset_counters(c, true)) return rc;
        HIPCHK(c, hipEventRecord(c->ev0, c->st));
        // verification mode: smaller launches, each followed by publishing its
        // new states (k_publish) and checking its deferred hits (k_verify)
        // SYMMETRY: every lane of a launch could defer a tied successor, so a
        // launch holds at most tie_cap / lanes states (5.6 M for S = 3, K = 4):
        // the tie buffer cannot overflow whatever the model's tie rate
        const u64 sym_chunk = c->sh.sym ? std::max<u64>(1, std::min<u64>(CHUNK, c->B.tie_cap / (u64)c->P.off[10])) : CHUNK;
        const u64 chunk = c->sh.verify ? (1ull << 20) : c->sh.sym ? sym_chunk : CHUNK;
        const u64 nlaunch = (hi - lo + chunk - 1) / chunk;
        const u64 even = (hi - lo + nlaunch - 1) / nlaunch;  // <= chunk
        for (u64 a = lo, b = 0; a < hi; a = b) {
            b = std::min(hi, a + even);
            if (c->spill.on && c->spill.dev_links) {
                // the ring window: [a, count) is live (the rest of the frontier and
                // the level being built); a state yields at most max_new_per_state
                // new states, so a launch of n states cannot overwrite a live state
                // when count + n * that <= a + win — nothing is ever moved
                const u64 lanes = max_new_per_state(c), count = c->h_ctr->count, win = c->spill.win;
                const u64 room = count - a < win ? a + win - count : 0;
                u64 want = std::min(b - a, room / lanes);
                if (c->sh.verify) want = std::min(want, c->B.hcap / lanes);  // hbuf holds every hit of a launch
                if (want == 0)
                    return fail(c, RMC_E_CAPACITY,
                                "spill: the device window (" + std::to_string(win) +
                                    " states) cannot hold the frontier and the level being built; raise "
                                    "rmc_config.device_window, or give the fingerprint set less HBM "
                                    "(rmc_config.set_bytes, rmc-tlc -fpmem: its " +
                                    std::to_string(c->table_slots) + " slots take " +
                                    std::to_string((c->table_slots * (c->sh.verify ? 16 : 8)) >> 30) +
                                    " GiB) so the window gets more");
                b = a + want;
                if (c->sh.verify) {
                    // the launch may overwrite the ring slots of states below
                    // count + n * lanes - win (<= a): copy them to the host first, and
                    // send hits on them to hbuf
                    const u64 top = count + want * lanes;
                    const u64 vlo = top > win ? top - win : 0;
                    if (int rc = verify_copy_out(c, vlo)) return rc;
                    c->B.vlo = vlo;
                }
            } else if (c->spill.on) {
                // a state yields at most max_new_per_state new states: a launch of
                // n states stays inside the window when n * that <= room.  Launches
                // shrink as the window fills; below 2^20 states the expanded
                // states [base, a) move to the host first — once they are at
                // least 1/8 of what the move shifts down (or nothing fits)
                const u64 lanes = max_new_per_state(c);
                const u64 count = c->h_ctr->count, fit = (c->B.cap - count) / lanes;
                u64 want = b - a;
                const u64 old = a - c->spill.base;
                const bool due = fit < std::min<u64>(want, 1ull << 20) && old && (old * 8 >= count - a || fit == 0);
                if (due)
                    if (int rc = spill_to(c, a, count)) return rc;
                want = std::min(want, (c->B.cap - count) / lanes);
                if (c->sh.verify) {
                    want = std::min(want, c->B.hcap / lanes);
                    c->B.vlo = c->spill.base;  // [0, base) were copied to the host by spill_to
                }
                if (want == 0)
                    return fail(c, RMC_E_CAPACITY,
                                "spill: the device window (" + std::to_string(c->spill.win) +
                                    " states) cannot hold the frontier and the level being built; raise "
                                    "rmc_config.device_window, or give the fingerprint set less HBM "
                                    "(rmc_config.set_bytes, rmc-tlc -fpmem: its " +
                                    std::to_string(c->table_slots) + " slots take " +
                                    std::to_string((c->table_slots * (c->sh.verify ? 16 : 8)) >> 30) +
                                    " GiB) so the window gets more");
                b = a + want;
            }
            HIPCHK(c, launch(c->sh, 0, c->P, c->PT, c->B, a, b, nullptr, nullptr, 0, nullptr, c->st));
            c->res.expand_launches += 1;
            if (c->sh.sym && !c->sh.verify) {
                HIPCHK(c, launch(c->sh, 10, c->P, c->PT, c->B, 0, 0, nullptr, nullptr, 0, nullptr, c->st));
                HIPCHK(c, hipMemsetAsync(&c->B.ctr->nties, 0, 8, c->st));
            }
            if (c->sh.verify) {
                const u64 before = c->h_ctr->count;
                if (int rc = read_counters(c)) return rc;
                if (c->h_ctr->overflow) break;
                HIPCHK(c, launch(c->sh, 5, c->P, c->PT, c->B, before, c->h_ctr->count, nullptr, nullptr, 0, nullptr,
                                 c->st));
                HIPCHK(c, launch(c->sh, 6, c->P, c->PT, c->B, c->h_ctr->vcount, 0, nullptr, nullptr, 0, nullptr,
                                 c->st));
                HIPCHK(c, hipMemsetAsync(&c->B.ctr->vcount, 0, 8, c->st));
                c->h_ctr->vcount = 0;
                if (c->h_ctr->hcount)  // hits on spilled owners: against their host copies
                    if (int rc = verify_host_hits(c, c->h_ctr->hcount)) return rc;
            }
            if (c->spill.on) {
                if (int rc = read_counters(c)) return rc;
                if (c->h_ctr->overflow || c->h_ctr->table_full) break;
                if (c->h_ctr->count > c->spill.total_cap)
                    return fail(c, RMC_E_CAPACITY, "spill: more states than rmc_config.state_capacity (" +
                                                       std::to_string(c->spill.total_cap) + ")");
                if (c->spill.dev_links) {  // the ring: states below count - win are overwritten
                    const u64 cnt = c->h_ctr->count, win = c->spill.win;
                    c->spill.base = cnt > win ? cnt - win : 0;
                    c->res.spilled = c->spill.base;
                    c->res.spills = cnt / win;  // passes of the ring
                }
            }
        }
        HIPCHK(c, hipEventRecord(c->ev1, c->st));
        if (int rc = read_counters(c)) return rc;
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->res.expand_kernel_seconds += 1e-3 * ms;
        const Counters& k = *c->h_ctr;
        if (k.table_full) return fail(c, RMC_E_CAPACITY, "fingerprint set full");
        if (k.overflow >> 8) return fail(c, RMC_E_CAPACITY, capacity_message(c, k.overflow, depth));
        if (k.overflow & 4u) return fail(c, RMC_E_CAPACITY, "verification buffer full");
        if (k.overflow & 16u) return fail(c, RMC_E_CAPACITY, "symmetry tie buffer full");
        if (k.overflow & 8u) return fail(c, RMC_E_HIP, "verification: a stored state has no fingerprint slot");
        c->res.collisions += k.collisions;
        c->res.verified += k.vchecked;
        if (k.overflow) {
            return fail(c, RMC_E_CAPACITY, "state store full (capacity " + std::to_string(c->B.cap) +
                                                " states); raise rmc_config.state_capacity");
        }
        c->res.generated += k.generated;
        c->res.probes += k.probes;
        c->walked += k.walked;
        const u64 nnew = k.count - hi;
        if (nnew) {
            ++depth;
            c->level_start.push_back(k.count);
        }
        c->res.distinct = k.count;
        if (k.viol != ~0ull) {
            c->res.violated_inv = 1 << (int)(k.viol & 15);
            c->res.violation_depth = depth;
            c->have_target = 1;
            c->target_idx = k.viol >> 4;
        } else if ((c->cfg.flags & RMC_FLAG_CHECK_DEADLOCK) && k.deadlock != ~0ull) {
            c->res.deadlock = 1;
            c->have_target = 1;
            c->target_idx = k.deadlock;
        }
        if (cb) {
            rmc_level_stats ls{};
            ls.level = nnew ? depth - 1 : depth;
            ls.generated = c->res.generated;
            ls.distinct = k.count;
            ls.new_states = nnew;
            ls.seconds = secs();
            if (cb(&ls, user)) {
                c->res.left_on_queue = nnew;
                break;
            }
        }
        if (!nnew) break;
    }
    c->res.distinct = c->level_start.back();
    c->res.depth = depth;
    c->res.verified_spilled = c->spill.host_hits;
    const double D = (double)c->res.distinct, G = (double)c->res.generated;
    // TLC's "calculated (optimistic)" fingerprint-collision estimate
    c->res.collision_probability = fp_collision_estimate(D, G, c->table_slots, c->set_epoch != 0);
    c->res.seconds = secs();
    // lane efficiency of the walk: enabled lanes / visited slots (the kernels count
    // the slots only when built with -DRMC_WALK_STATS_BUILD: a register in the hot loop)
    if (getenv("RMC_WALK_STATS"))
        fprintf(stderr, "[rmc] lane walk: %llu slots visited, %llu generated, %llu probes: efficiency %.4f\n",
                (unsigned long long)c->walked, (unsigned long long)c->res.generated,
                (unsigned long long)c->res.probes, c->walked ? G / (double)c->walked : 0.0);
    return 0;
}

int rmc_set_seed(rmc_ctx* c, uint64_t seed) {
    if (!c) return RMC_E_INVAL;
    c->cfg.seed = seed;
    return 0;
}

int rmc_set_fp_bits(rmc_ctx* c, int32_t bits) {
    if (!c || bits < 1 || bits > 64) return RMC_E_INVAL;
    if (!c->sh.verify) return fail(c, RMC_E_INVAL, "rmc_set_fp_bits needs RMC_FLAG_VERIFY_STATES");
    c->P.fp_mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
    return 0;
}

int rmc_get_result(const rmc_ctx* c, rmc_result* out) {
    if (!c || !out) return RMC_E_INVAL;
    *out = c->res;
    return 0;
}

// ---- checkpoint / recovery (TLC -checkpoint / -recover) ------------------------
// File: header, level boundaries, then the stored states, parent refs and lanes
// of levels 1..depth.  The fingerprint set is not written: rmc_recover rebuilds
// it from the states (k_rehash), one pass over the store.
namespace {
// The header embeds the ABI structs rmc_config and rmc_result, so its size is
// written too and must match: a struct that grows changes kCkptVersion.
constexpr uint32_t kCkptVersion = 5;  // 3: rmc_result with parked / exchange_wait_seconds; 4: the set holds
                                      // k ^ s values (raft_packed.h Fp), rmc_result with spill_links_on_device;
                                      // 5: rmc_config.set_bytes, rmc_result.verified_spilled
struct CkptHeader {
    char magic[8];
    uint32_t version, nw;
    uint32_t header_bytes, pad_;
    rmc_config cfg;
    uint64_t count, nlevels;
    int32_t depth;
    int32_t shard;   // sharded checkpoint: rank | world << 16 (0: single GPU)
    rmc_result res;
    uint64_t first;  // states are written from this index on (0: all; else the frontier)
    uint64_t slots;  // fingerprint-set slots dumped after the states (first > 0), else 0
};
const char kCkptMagic[8] = {'R', 'M', 'C', 'C', 'K', 'P', 'T', '1'};

bool same_model(const rmc_config& a, const rmc_config& b) {
    return a.n_servers == b.n_servers && a.n_values == b.n_values && a.max_term == b.max_term &&
           a.max_log_len == b.max_log_len && a.max_msgs == b.max_msgs && a.max_dup == b.max_dup &&
           ((a.flags ^ b.flags) & ~RMC_FLAG_SPILL) == 0 && a.invariants == b.invariants && a.seed == b.seed;
}

// Copy n bytes between a device buffer and a file through a pinned bounce buffer.
int move_file(rmc_ctx* c, FILE* f, void* dev, u64 n, bool to_file) {
    const u64 B = 64ull << 20;
    void* h = nullptr;
    HIPCHK(c, hipHostMalloc(&h, B, hipHostMallocDefault));
    int rc = 0;
    for (u64 off = 0; off < n && !rc; off += B) {
        const u64 k = std::min(B, n - off);
        char* d = (char*)dev + off;
        if (to_file) {
            if (hipMemcpy(h, d, k, hipMemcpyDeviceToHost) != hipSuccess) rc = RMC_E_HIP;
            else if (fwrite(h, 1, k, f) != k) rc = fail(c, RMC_E_IO, "checkpoint write failed");
        } else {
            if (fread(h, 1, k, f) != k) rc = fail(c, RMC_E_IO, "checkpoint file truncated");
            else if (hipMemcpy(d, h, k, hipMemcpyHostToDevice) != hipSuccess) rc = RMC_E_HIP;
        }
    }
    (void)hipHostFree(h);
    if (rc == RMC_E_HIP) return fail(c, rc, "checkpoint copy failed");
    return rc;
}
}  // namespace

// Layout: header, level table, parent[0, count), act[0, count), store[first,
// count), then — when the states below `first` have spilled and no longer
// exist — the fingerprint set itself (TLC checkpoints its FPSet too).
int rmc_checkpoint(rmc_ctx* c, const char* path) {
    if (!c || !path) return RMC_E_INVAL;
    if (c->wide) return fail(c, RMC_E_STATE, "checkpoint / recover: not supported on the wide layout");
    if (c->level_start.size() < 2 || c->have_target)
        return fail(c, RMC_E_STATE, "checkpoint: needs a BFS stopped at a level boundary without a violation");
    if (c->res.left_on_queue == 0) return fail(c, RMC_E_STATE, "checkpoint: the search is complete");
    if (c->spill.on && c->sh.verify)
        return fail(c, RMC_E_STATE, "checkpoint: not supported with RMC_FLAG_VERIFY_STATES and RMC_FLAG_SPILL "
                                    "(the host copies of the spilled states are not written)");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    HIPCHK(c, hipStreamSynchronize(c->st));
    // a sharded search: every rank writes its own part, <path>.rank<r> (collective
    // only in the sense that every rank calls it; the global counts ride in res)
    const std::string file = shard_path(c, path);
    FILE* f = fopen(file.c_str(), "wb");
    if (!f) return fail(c, RMC_E_IO, "checkpoint: cannot create " + file);
    CkptHeader h{};
    h.shard = c->dist.on ? (c->dist.rank | (c->dist.world << 16)) : 0;
    memcpy(h.magic, kCkptMagic, 8);
    h.version = kCkptVersion;
    h.header_bytes = (uint32_t)sizeof(CkptHeader);
    h.nw = (uint32_t)c->NW;
    h.cfg = c->cfg;
    h.count = c->level_start.back();
    h.nlevels = c->level_start.size();
    h.depth = c->res.depth;
    h.res = c->res;
    const u64 base = c->spill.on ? c->spill.base : 0;
    h.first = base ? c->level_start[h.nlevels - 2] : 0;  // >= base at a level boundary
    h.slots = base ? c->table_slots : 0;
    h.pad_ = h.slots ? c->set_epoch : 0;  // the dumped set's epoch tag (0: untagged)
    int rc = fwrite(&h, sizeof h, 1, f) == 1 && fwrite(c->level_start.data(), 8, h.nlevels, f) == h.nlevels
                 ? 0 : fail(c, RMC_E_IO, "checkpoint write failed");
    auto put = [&](const void* p, u64 n) {
        if (!rc && n && fwrite(p, 1, n, f) != n) rc = fail(c, RMC_E_IO, "checkpoint write failed");
    };
    const u64 lb = c->spill.dev_links ? 0 : base;  // links below lb are on the host
    const u64 nd = h.count - lb;
    if (lb) put(c->spill.h_parent, lb * 8);
    if (!rc) rc = move_file(c, f, c->B.parent + lb, nd * 8, true);
    if (lb) put(c->spill.h_act, lb);
    if (!rc) rc = move_file(c, f, c->B.act + lb, nd, true);
    for (u64 i = h.first; !rc && i < h.count;) {  // the ring window: in up to two pieces
        const u64 sl = wslot(c->B, i), n = std::min(h.count - i, c->B.wmask == ~0ull ? h.count - i : c->spill.win - sl);
        rc = move_file(c, f, c->B.store + sl * (u64)c->NW, n * (u64)c->NW * 4, true);
        i += n;
    }
    if (!rc && h.slots) rc = move_file(c, f, c->B.table, h.slots * 8, true);
    if (fclose(f) != 0 && !rc) rc = fail(c, RMC_E_IO, "checkpoint close failed");
    return rc;
}

int rmc_recover(rmc_ctx* c, const char* path) {
    if (!c || !path) return RMC_E_INVAL;
    if (c->wide) return fail(c, RMC_E_STATE, "checkpoint / recover: not supported on the wide layout");
    if (c->spill.on && c->sh.verify)
        return fail(c, RMC_E_STATE, "recover: not supported with RMC_FLAG_VERIFY_STATES and RMC_FLAG_SPILL");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    const std::string file = shard_path(c, path);
    FILE* f = fopen(file.c_str(), "rb");
    if (!f) return fail(c, RMC_E_IO, "recover: cannot open " + file);
    CkptHeader h{};
    int rc = 0;
    std::vector<u64> ls;
    // the fixed prefix first (magic, version): an older version is refused by
    // name before its differently laid-out remainder is interpreted
    const size_t pre = offsetof(CkptHeader, header_bytes);
    if (fread(&h, pre, 1, f) != 1 || memcmp(h.magic, kCkptMagic, 8) != 0)
        rc = fail(c, RMC_E_IO, "recover: not an rmc checkpoint");
    else if (h.version != kCkptVersion)
        rc = fail(c, RMC_E_IO, "recover: checkpoint format version " + std::to_string(h.version) +
                                   " (this build reads version " + std::to_string(kCkptVersion) +
                                   "); recreate the checkpoint with this build");
    else if (fread((char*)&h + pre, sizeof h - pre, 1, f) != 1 || h.header_bytes != (uint32_t)sizeof(CkptHeader))
        rc = fail(c, RMC_E_IO, "recover: checkpoint header truncated or of another layout");
    else if (h.shard != (c->dist.on ? (c->dist.rank | (c->dist.world << 16)) : 0))
        rc = fail(c, RMC_E_INVAL, "recover: the checkpoint is of another shard layout (rank / world), or of a "
                                  "single-GPU run recovered on a sharded ctx or the reverse");
    else if (h.nw != (uint32_t)c->NW || !same_model(h.cfg, c->cfg))
        rc = fail(c, RMC_E_INVAL, "recover: the checkpoint is of another model (constants, bounds, flags or seed)");
    else if (h.first && (!c->spill.on || h.slots != c->table_slots))
        rc = fail(c, RMC_E_INVAL, "recover: a spilled checkpoint holds the fingerprint set, not the spilled "
                                  "states; recover it with RMC_FLAG_SPILL and the same state_capacity");
    else {
        ls.resize(h.nlevels);
        if (h.nlevels < 2 || fread(ls.data(), 8, h.nlevels, f) != h.nlevels || ls.back() != h.count ||
            h.first > h.count)
            rc = fail(c, RMC_E_IO, "recover: corrupt level table");
    }
    // states [0, s) keep only their trace links, on the host (spill mode, when
    // they do not all fit the window); [s, count) — at least the frontier — go
    // to the device
    u64 s = 0;
    if (!rc) {
        s = h.first ? h.first : (c->spill.on && h.count > c->spill.win) ? ls[ls.size() - 2] : 0;
        const u64 room = c->spill.on ? c->spill.win : c->B.cap;
        if (h.count - s > room || (c->spill.on && h.count > c->spill.total_cap))
            rc = fail(c, RMC_E_CAPACITY, "recover: the checkpoint holds more states than this ctx's capacity");
        if (!rc && !h.first && s && h.count - s >= room)  // no room left to stream the rehash through
            rc = fail(c, RMC_E_CAPACITY, "recover: the frontier fills the device window");
    }
    if (rc) {
        fclose(f);
        return rc;
    }
    if (c->spill.on) {
        if (c->spill.ahead.joinable()) c->spill.ahead.join();  // it may be touching [0, s)
        spill_rebase(c, 0);
        if (!c->spill.dev_links) c->spill.faulted = std::max(c->spill.faulted, s);  // fread backs the links it writes
    }
    const u64 NW = (u64)c->NW, W = NW * 4;
    u32* dstore = c->spill.on ? c->spill.store : c->B.store;
    u64* dparent = c->spill.on ? c->spill.parent : c->B.parent;
    uint8_t* dact = c->spill.on ? c->spill.act : c->B.act;
    auto get = [&](void* p, u64 n) {
        if (!rc && n && fread(p, 1, n, f) != n) rc = fail(c, RMC_E_IO, "checkpoint file truncated");
    };
    HIPCHK(c, launch_fill(c->B.table, c->table_slots * 8, 0, c->st));
    if (c->sh.verify) HIPCHK(c, launch_fill(c->B.sidx, c->table_slots * 8, 0xFF, c->st));
    // footprints are not checkpointed: the recovered frontier is expanded without
    // diamond skipping (FOOT_VALID clear), the levels after it with
    HIPCHK(c, hipMemsetAsync(c->spill.on ? c->spill.foot : c->B.foot, 0,
                             (c->spill.on ? c->spill.win : c->B.cap) * 8, c->st));
    // a dumped set keeps its entries' epoch tag (header pad_); states rehashed
    // below go into an untagged set
    c->set_epoch = h.slots ? std::min<u32>(h.pad_, 255u) : 0u;
    HIPCHK(c, set_fp_salt(c->sh, c->cfg.seed, c->set_epoch, c->st));
    if (int r2 = reset_counters(c, false)) return r2;
    const u64 ls0 = c->spill.dev_links ? 0 : s;  // links below ls0 go to the host
    if (ls0) get(c->spill.h_parent, ls0 * 8);
    if (!rc) rc = move_file(c, f, dparent, (h.count - ls0) * 8, false);
    if (ls0) get(c->spill.h_act, ls0);
    if (!rc) rc = move_file(c, f, dact, h.count - ls0, false);
    if (!h.first && s && !rc) {
        // no set in the file: rehash the states below s through the free part
        // of the window (the frontier is loaded after them, at its start)
        const u64 piece = c->spill.win - (h.count - s);
        u32* area = dstore + (h.count - s) * NW;
        for (u64 p = 0; p < s && !rc; p += piece) {
            const u64 k = std::min(piece, s - p);
            rc = move_file(c, f, area, k * W, false);
            DevBufs T = c->B;
            T.store = (u32*)((uintptr_t)area - (uintptr_t)(p * W));
            T.wmask = ~0ull;  // indexed through the biased pointer, not the ring
            if (!rc) HIPCHK(c, launch(c->sh, 7, c->P, c->PT, T, p, p + k, nullptr, nullptr, 0, nullptr, c->st));
            if (!rc) HIPCHK(c, hipStreamSynchronize(c->st));
        }
    }
    if (c->spill.on && c->spill.dev_links) {  // the ring window: state i at slot i & wmask
        const u64 win = c->spill.win;
        for (u64 i = s; !rc && i < h.count;) {
            const u64 sl = i & (win - 1), n = std::min(h.count - i, win - sl);
            rc = move_file(c, f, dstore + sl * NW, n * W, false);
            i += n;
        }
    } else if (!rc) {
        rc = move_file(c, f, dstore, (h.count - s) * W, false);
    }
    if (!rc && h.slots) rc = move_file(c, f, c->B.table, h.slots * 8, false);
    fclose(f);
    if (rc) return rc;
    if (s) spill_rebase(c, s);
    if (!h.slots) HIPCHK(c, launch(c->sh, 7, c->P, c->PT, c->B, s, h.count, nullptr, nullptr, 0, nullptr, c->st));
    if (c->sh.verify) HIPCHK(c, launch(c->sh, 5, c->P, c->PT, c->B, 0, h.count, nullptr, nullptr, 0, nullptr, c->st));
    if (int r2 = read_counters(c)) return r2;
    if (c->h_ctr->table_full) return fail(c, RMC_E_CAPACITY, "recover: fingerprint set full");
    if (c->h_ctr->overflow) return fail(c, RMC_E_IO, "recover: the checkpoint holds duplicate states");
    c->level_start = ls;
    c->res = h.res;
    c->resume = 1;
    c->resume_depth = h.depth;
    return 0;
}

// The counterexample: parent links back to Init, then the states.  States
// whose store was spilled are re-derived by replaying the recorded lanes from
// the last state still known (Init at worst) with the listing kernel — the
// stored successor of a parent through a lane is exactly what it lists.
int rmc_trace(rmc_ctx* c, rmc_state_view* states, int32_t* families, int32_t* instances, size_t cap, size_t* len) {
    if (!c || !len) return RMC_E_INVAL;
    if (!c->have_target) return fail(c, RMC_E_STATE, "no violation or deadlock to trace");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (c->wide) return trace_wide(c, states, families, instances, cap, len);
    if (c->dist.on) return trace_sharded(c, states, families, instances, cap, len);
    std::vector<u64> chain;
    std::vector<uint8_t> acts;
    u64 idx = c->target_idx;
    for (;;) {
        u64 p = 0;
        uint8_t a = 0;
        if (int rc = read_link(c, idx, &p, &a)) return rc;
        chain.push_back(idx);
        acts.push_back(a);
        if (p == ~0ull || chain.size() > 100000) break;
        idx = p;
    }
    std::reverse(chain.begin(), chain.end());
    std::reverse(acts.begin(), acts.end());
    *len = chain.size();
    const u64 NW = (u64)c->NW, RW = 6 + NW, lanes = (u64)c->P.off[10];
    std::vector<u32> cur(NW);
    u32 *d_in = nullptr, *d_out = nullptr;
    unsigned long long* d_cnt = nullptr;
    int rc = 0;
    for (size_t q = 0; q < chain.size() && !rc; ++q) {
        if (!c->spill.on || chain[q] >= c->spill.base) {
            HIPCHK(c, hipMemcpy(cur.data(), c->B.store + wslot(c->B, chain[q]) * NW, NW * 4, hipMemcpyDeviceToHost));
        } else if (q == 0) {  // Init (raft.tla:125-129), the one initial state
            rmc_state_view iv;
            init_view(c->cfg, &iv);
            std::string why;
            if (encode_view(c, iv, cur.data(), &why)) return fail(c, RMC_E_INVAL, why);
        } else {  // replay lane acts[q] from the previous state on the device
            if (!d_in) {
                if (hipMalloc(&d_in, NW * 4) != hipSuccess || hipMalloc(&d_out, lanes * RW * 4) != hipSuccess ||
                    hipMalloc(&d_cnt, 8) != hipSuccess)
                    rc = fail(c, RMC_E_NOMEM, "trace: replay buffers");
            }
            std::vector<u32> recs(lanes * RW);
            unsigned long long n = 0;
            if (!rc && (hipMemcpy(d_in, cur.data(), NW * 4, hipMemcpyHostToDevice) != hipSuccess ||
                        hipMemset(d_cnt, 0, 8) != hipSuccess ||
                        launch(c->sh, 2, c->P, c->PT, c->B, 1, 0, d_in, d_out, lanes, d_cnt, c->st) != hipSuccess ||
                        hipStreamSynchronize(c->st) != hipSuccess ||
                        hipMemcpy(&n, d_cnt, 8, hipMemcpyDeviceToHost) != hipSuccess ||
                        hipMemcpy(recs.data(), d_out, std::min<u64>(n, lanes) * RW * 4, hipMemcpyDeviceToHost) != hipSuccess))
                rc = fail(c, RMC_E_HIP, "trace: replay launch failed");
            bool found = false;
            for (u64 r = 0; !rc && r < std::min<u64>(n, lanes); ++r) {
                const u32* rec = &recs[r * RW];
                if (rec[2] == acts[q] && rec[3]) {
                    memcpy(cur.data(), rec + 6, NW * 4);
                    found = true;
                    break;
                }
            }
            if (!rc && !found) rc = fail(c, RMC_E_STATE, "trace: a recorded lane is not enabled on replay");
        }
        if (!rc && q < cap) {
            if (states) decode_state(c, cur.data(), &states[q]);
            if (families) families[q] = family_of(c->P, acts[q]);
            if (instances) instances[q] = acts[q] == 255 ? -1 : acts[q];
        }
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    (void)hipFree(d_cnt);
    return rc;
}

}  // extern "C"

// ---- simulation: SmokeInit sampler (Smokeraft.tla:4-76) and random walks -------
namespace {

// RandomSubset(k, X): k distinct random elements of X, X given by a sampler.
template <class T, class F>
std::vector<T> random_subset(int k, F draw, std::mt19937_64& g) {
    std::vector<T> out;
    for (int guard = 0; (int)out.size() < k && guard < 100000; ++guard) {
        T x = draw(g);
        if (std::find(out.begin(), out.end(), x) == out.end()) out.push_back(x);
    }
    return out;
}

struct SmokeDomains {
    int S, V, nat;
    int uni(std::mt19937_64& g, int lo, int hi) const {  // uniform in lo..hi
        return lo + (int)(g() % (u64)(hi - lo + 1));
    }
    // BoundedSeq([term : SmokeNat, value : Value], n) (Smokeraft.tla:4-6): uniform over
    // the whole set of sequences of length 0..n; encoded as (len, e0, e1, ...).
    std::vector<int> seq(std::mt19937_64& g, int n) const {
        const u64 E = (u64)(nat + 1) * (u64)V;
        u64 total = 0, p = 1;
        for (int m = 0; m <= n; ++m, p *= E) total += p;
        u64 r = g() % total;
        int len = 0;
        p = 1;
        while (r >= p) { r -= p; p *= E; ++len; }
        std::vector<int> s{len};
        for (int x = 0; x < len; ++x) {
            const u64 e = r % E;
            r /= E;
            s.push_back((int)(e / (u64)V));  // term
            s.push_back((int)(e % (u64)V));  // value
        }
        return s;
    }
};

// One message of SmokeMessageType (Smokeraft.tla:24-62) as a canonical int vector.
std::vector<int> smoke_msg(const SmokeDomains& D, int type, std::mt19937_64& g) {
    std::vector<int> v{type, D.uni(g, 0, D.nat), D.uni(g, 0, D.S - 1), D.uni(g, 0, D.S - 1)};
    if (type == RVQ) { v.push_back(D.uni(g, 0, D.nat)); v.push_back(D.uni(g, 0, D.nat)); }
    if (type == AEQ) {
        v.push_back(D.uni(g, -1, 1));              // mprevLogIndex \in SmokeInt
        v.push_back(D.uni(g, 0, D.nat));           // mprevLogTerm
        const auto e = D.seq(g, 1);                // mentries \in SmokeSeq(...)
        v.insert(v.end(), e.begin(), e.end());
        v.push_back(D.uni(g, 0, D.nat));           // mcommitIndex
    }
    if (type == RVP) {
        v.push_back(D.uni(g, 0, 1));               // mvoteGranted \in BOOLEAN
        const auto e = D.seq(g, 1);                // mlog \in SmokeSeq(...)
        v.insert(v.end(), e.begin(), e.end());
    }
    if (type == AEP) { v.push_back(D.uni(g, 0, 1)); v.push_back(D.uni(g, 0, D.nat)); }
    return v;
}

void msg_to_view(const std::vector<int>& v, rmc_msg_view* m) {
    memset(m, 0, sizeof *m);
    m->mtype = v[0];
    m->mterm = v[1];
    m->msource = v[2];
    m->mdest = v[3];
    m->count = 1;
    size_t p = 4;
    auto seq = [&](rmc_entry* out, int32_t* len) {
        *len = v[p++];
        for (int x = 0; x < *len; ++x) { out[x].term = v[p++]; out[x].value = v[p++]; }
    };
    if (v[0] == RVQ) { m->mlastLogTerm = v[p++]; m->mlastLogIndex = v[p++]; }
    if (v[0] == AEQ) { m->mprevLogIndex = v[p++]; m->mprevLogTerm = v[p++]; seq(m->mentries, &m->mentries_len); m->mcommitIndex = v[p++]; }
    if (v[0] == RVP) { m->mvoteGranted = v[p++]; seq(m->mlog, &m->mlog_len); }
    if (v[0] == AEP) { m->msuccess = v[p++]; m->mmatchIndex = v[p++]; }
}

// SmokeInit (Smokeraft.tla:64-76): k choices for each of the 9 per-server
// variables, all k^9 combinations, each with the same bag of k messages drawn as
// [RandomSubset(k, SmokeMessageType) -> {1}].
}  // namespace

namespace rmc_host {
// SmokeInit (Smokeraft.tla:64-76) as k^9 views, in RandomSubset product order.
int smoke_views(const rmc_ctx* c, const rmc_sim_config& sc, std::vector<rmc_state_view>* views, std::string* why) {
    const int S = c->cfg.n_servers, k = sc.smoke_k;
    SmokeDomains D{S, c->cfg.n_values, sc.smoke_nat > 0 ? sc.smoke_nat : 2};
    if (D.nat > 3 && !c->wide) { *why = "smoke_nat > 3 exceeds the packed index range"; return RMC_E_INVAL; }
    if (D.nat > 100) { *why = "smoke_nat > 100"; return RMC_E_INVAL; }
    const int bag = c->wide ? rmc::wide::KW : c->sh.K;
    if (k > bag) { *why = "smoke_k messages exceed the bag capacity (set MaxMsgs >= k)"; return RMC_E_INVAL; }
    std::mt19937_64 g(sc.seed ^ 0x5350AC3ull);
    using V = std::vector<int>;
    auto fn = [&](auto elem) { return [&, elem](std::mt19937_64& gg) { V v; for (int i = 0; i < S; ++i) { auto e = elem(gg); v.insert(v.end(), e.begin(), e.end()); } return v; }; };
    auto one = [&](int lo, int hi) { return [&D, lo, hi](std::mt19937_64& gg) { return V{D.uni(gg, lo, hi)}; }; };
    const auto ct = random_subset<V>(k, fn(one(0, D.nat)), g);                               // :67
    const auto st = random_subset<V>(k, fn(one(0, 2)), g);                                   // :68
    const auto vf = random_subset<V>(k, fn(one(-1, S - 1)), g);                              // :69 (Nil = -1)
    const auto lg = random_subset<V>(k, fn([&](std::mt19937_64& gg) { return D.seq(gg, 3); }), g);  // :70
    const auto ci = random_subset<V>(k, fn(one(0, D.nat)), g);                               // :71
    const auto vr = random_subset<V>(k, fn(one(0, (1 << S) - 1)), g);                        // :72
    const auto vg = random_subset<V>(k, fn(one(0, (1 << S) - 1)), g);                        // :73
    auto row = [&](int lo, int hi) { return [&, lo, hi](std::mt19937_64& gg) { V v; for (int j = 0; j < S; ++j) v.push_back(D.uni(gg, lo, hi)); return v; }; };
    const auto ni = random_subset<V>(k, fn(row(1, D.nat)), g);                               // :74
    const auto mi = random_subset<V>(k, fn(row(0, D.nat)), g);                               // :75
    std::vector<V> mtype_union;                                                              // :58-62
    for (int t : {RVQ, AEQ, RVP, AEP}) {
        auto part = random_subset<V>(k, [&, t](std::mt19937_64& gg) { return smoke_msg(D, t, gg); }, g);
        mtype_union.insert(mtype_union.end(), part.begin(), part.end());
    }
    const auto msgs = random_subset<V>(k, [&](std::mt19937_64& gg) { return mtype_union[gg() % mtype_union.size()]; }, g);  // :76
    for (const auto* vec : {&ct, &st, &vf, &lg, &ci, &vr, &vg, &ni, &mi})
        if ((int)vec->size() != k) { *why = "RandomSubset could not draw k distinct elements"; return RMC_E_INVAL; }
    u64 n = 1;
    for (int x = 0; x < 9; ++x) n *= (u64)k;
    views->assign(n, rmc_state_view{});
    for (u64 idx = 0; idx < n; ++idx) {
        int dg[9];
        u64 r = idx;
        for (int x = 0; x < 9; ++x) { dg[x] = (int)(r % (u64)k); r /= (u64)k; }
        rmc_state_view v;
        memset(&v, 0, sizeof v);
        v.n_servers = S;
        size_t lp = 0;
        for (int i = 0; i < S; ++i) {
            v.currentTerm[i] = ct[dg[0]][i];
            v.state[i] = st[dg[1]][i];
            v.votedFor[i] = vf[dg[2]][i];
            v.commitIndex[i] = ci[dg[4]][i];
            v.votesResponded[i] = (uint32_t)vr[dg[5]][i];
            v.votesGranted[i] = (uint32_t)vg[dg[6]][i];
            for (int j = 0; j < S; ++j) {
                v.nextIndex[i][j] = ni[dg[7]][i * S + j];
                v.matchIndex[i][j] = mi[dg[8]][i * S + j];
            }
        }
        const V& L = lg[dg[3]];
        for (int i = 0; i < S; ++i) {
            v.log_len[i] = L[lp++];
            for (int x = 0; x < v.log_len[i]; ++x) { v.log[i][x].term = L[lp++]; v.log[i][x].value = L[lp++]; }
        }
        v.n_msgs = (int)msgs.size();
        for (size_t q = 0; q < msgs.size(); ++q) msg_to_view(msgs[q], &v.msgs[q]);
        (*views)[idx] = v;
    }
    return 0;
}
}  // namespace rmc_host

namespace {
int smoke_init(const rmc_ctx* c, const rmc_sim_config& sc, std::vector<u32>* packed, std::string* why) {
    std::vector<rmc_state_view> views;
    if (int rc = smoke_views(c, sc, &views, why)) return rc;
    packed->assign(views.size() * (u64)c->NW, 0u);
    for (size_t q = 0; q < views.size(); ++q)
        if (int rc = encode_view(c, views[q], packed->data() + q * (u64)c->NW, why)) return rc;
    return 0;
}

int run_sim(rmc_ctx* c, const rmc_sim_config* sc, rmc_sim_result* out, i64 rec_beh, std::vector<u32>* rec,
            std::vector<rmc_state_view>* wrec = nullptr) {
    if (!c || !sc || !out || sc->behaviours == 0 || sc->depth < 1 ||
        (sc->mode != RMC_SIM_WITHIN_CAPACITY && sc->mode != RMC_SIM_TRUNCATE && sc->mode != RMC_SIM_TLC))
        return RMC_E_INVAL;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    if (c->wide) return sim_wide(c, sc, out, rec_beh, wrec);
    if (sc->mode == RMC_SIM_TLC)
        return fail(c, RMC_E_INVAL, "RMC_SIM_TLC draws on the wide layout only (bounds beyond the packed capacity)");
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<u32> inits;
    std::string why;
    if (sc->smoke_k > 0) {
        if (int rc = smoke_init(c, *sc, &inits, &why)) return fail(c, rc, why);
    } else {
        rmc_state_view iv;
        init_view(c->cfg, &iv);
        inits.assign((size_t)c->NW, 0u);
        if (int rc = encode_view(c, iv, inits.data(), &why)) return fail(c, rc, why);
    }
    const u64 n_init = inits.size() / (u64)c->NW;
    // The model's bounds, as TLC's simulator respects a state CONSTRAINT; a
    // simulation model without one gets the packed capacity from the front-end
    // (rmc_model_from_files with RMC_FRONT_SIMULATE), so walks never exceed
    // what a state can hold.
    Params P = c->P;
    P.max_msgs = std::min(P.max_msgs, c->sh.K);
    u32 *d_init = nullptr, *d_rec = nullptr;
    SimCounters* d_out = nullptr;
    HIPCHK(c, hipMalloc(&d_init, inits.size() * 4));
    HIPCHK(c, hipMalloc(&d_out, sizeof(SimCounters)));
    if (rec) HIPCHK(c, hipMalloc(&d_rec, (size_t)sc->depth * c->NW * 4));
    SimCounters h{};
    h.viol = ~0ull;
    HIPCHK(c, hipMemcpy(d_init, inits.data(), inits.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(d_out, &h, sizeof h, hipMemcpyHostToDevice));
    HIPCHK(c, hipEventRecord(c->ev0, c->st));
    HIPCHK(c, launch_sim(c->sh, P, d_init, n_init, sc->behaviours, sc->depth, sc->seed, sc->mode, d_out, rec_beh, d_rec, c->st));
    HIPCHK(c, hipEventRecord(c->ev1, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    HIPCHK(c, hipMemcpy(&h, d_out, sizeof h, hipMemcpyDeviceToHost));
    if (rec) {
        rec->assign((size_t)(h.steps + 1) * c->NW, 0u);
        HIPCHK(c, hipMemcpy(rec->data(), d_rec, rec->size() * 4, hipMemcpyDeviceToHost));
    }
    (void)hipFree(d_init);
    (void)hipFree(d_out);
    (void)hipFree(d_rec);
    memset(out, 0, sizeof *out);
    out->behaviours = rec ? 1 : sc->behaviours;
    out->steps = h.steps;
    out->init_states = n_init;
    out->truncated = h.truncated;
    out->deadlocked = h.deadlocked;
    if (h.viol != ~0ull) {
        out->violated_inv = 1 << (int)((h.viol >> 40) & 15);
        out->violation_depth = (int32_t)(h.viol >> 44);
        out->violation_behaviour = h.viol & ((1ull << 40) - 1);
    }
    out->kernel_seconds = 1e-3 * ms;
    out->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

}  // namespace

extern "C" {

int rmc_simulate(rmc_ctx* c, const rmc_sim_config* sc, rmc_sim_result* out) { return run_sim(c, sc, out, -1, nullptr); }

int rmc_smoke_init(const rmc_config* cfg, const rmc_sim_config* sc, rmc_state_view* states, size_t cap, size_t* n) {
    if (!cfg || !sc || !n || sc->smoke_k < 1) return RMC_E_INVAL;
    std::string why;
    if (validate(cfg, &why)) return RMC_E_INVAL;
    rmc_ctx host;  // codec only: no device, no allocation
    host.cfg = *cfg;
    fill_params(&host);
    if (host.wide) {
        std::vector<rmc_state_view> views;
        if (smoke_views(&host, *sc, &views, &why)) return RMC_E_INVAL;
        *n = views.size();
        for (size_t q = 0; q < *n && q < cap && states; ++q) states[q] = views[q];
        return 0;
    }
    std::vector<u32> packed;
    if (smoke_init(&host, *sc, &packed, &why)) return RMC_E_INVAL;
    *n = packed.size() / (size_t)host.NW;
    for (size_t q = 0; q < *n && q < cap && states; ++q) decode_state(&host, packed.data() + q * host.NW, &states[q]);
    return 0;
}

int rmc_sim_replay(rmc_ctx* c, const rmc_sim_config* sc, uint64_t behaviour, rmc_state_view* states, size_t cap,
                   size_t* len) {
    if (!c || !sc || !len || behaviour >= sc->behaviours) return RMC_E_INVAL;
    rmc_sim_result r;
    std::vector<u32> rec;
    if (c->wide) {
        std::vector<rmc_state_view> wrec;
        if (int rc = run_sim(c, sc, &r, (i64)behaviour, nullptr, &wrec)) return rc;
        *len = wrec.size();
        for (size_t q = 0; q < *len && q < cap; ++q) states[q] = wrec[q];
        return 0;
    }
    if (int rc = run_sim(c, sc, &r, (i64)behaviour, &rec)) return rc;
    *len = rec.size() / (size_t)c->NW;
    for (size_t q = 0; q < *len && q < cap; ++q) decode_state(c, rec.data() + q * c->NW, &states[q]);
    return 0;
}

int rmc_probe_bench(int device, uint64_t table_bytes, uint64_t accesses, int mode, double* per_second) {
    if (!per_second || table_bytes < 4096 || accesses == 0 || (mode != 0 && mode != 1)) return RMC_E_INVAL;
    if (hipSetDevice(device) != hipSuccess) return RMC_E_NOGPU;
    u64 slots = 1;
    while (slots * 2 * 8 <= table_bytes) slots <<= 1;
    u64* table = nullptr;
    u64* sink = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = 0;
    const u64 threads = 256ull * 2048;                       // 8 blocks of 256 per CU
    const u32 iters = (u32)std::max<u64>(1, accesses / (threads * 8));
    float ms = 0.f;
    if (hipMalloc(&table, slots * 8) != hipSuccess || hipMalloc(&sink, 8) != hipSuccess) { rc = RMC_E_NOMEM; goto out; }
    if (hipStreamCreate(&st) != hipSuccess || hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
        rc = RMC_E_HIP;
        goto out;
    }
    if (hipMemsetAsync(table, 0, slots * 8, st) != hipSuccess) { rc = RMC_E_HIP; goto out; }
    // warm-up launch (page mapping, clocks), then the timed one
    if (launch_probe_bench(table, slots - 1, threads, 1, mode, sink, st) != hipSuccess) { rc = RMC_E_HIP; goto out; }
    if (hipEventRecord(e0, st) != hipSuccess) { rc = RMC_E_HIP; goto out; }
    if (launch_probe_bench(table, slots - 1, threads, iters, mode, sink, st) != hipSuccess) { rc = RMC_E_HIP; goto out; }
    if (hipEventRecord(e1, st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
        rc = RMC_E_HIP;
        goto out;
    }
    *per_second = (double)threads * 8.0 * iters / (1e-3 * ms);
out:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    (void)hipFree(table);
    (void)hipFree(sink);
    return rc;
}

int rmc_expand(rmc_ctx* c, const rmc_state_view* states, size_t n, rmc_succ_view* out, size_t cap, size_t* n_out) {
    if (!c || (!states && n) || !n_out) return RMC_E_INVAL;
    HIPCHK(c, hipSetDevice(c->cfg.device));
    *n_out = 0;
    if (n == 0) return 0;
    if (c->wide) return expand_wide(c, states, n, out, cap, n_out);
    const int NW = c->NW, RW = 6 + NW;
    std::vector<u32> packed(n * (size_t)NW);
    std::string why;
    for (size_t t = 0; t < n; ++t)
        if (encode_view(c, states[t], packed.data() + t * NW, &why))
            return fail(c, RMC_E_INVAL, "state " + std::to_string(t) + ": " + why);
    const u64 lanes = (u64)c->P.off[10];
    const u64 rcap = std::max<u64>(1, std::min<u64>((u64)cap, n * lanes));
    u32 *d_in = nullptr, *d_out = nullptr;
    unsigned long long* d_cnt = nullptr;
    HIPCHK(c, hipMalloc(&d_in, packed.size() * 4));
    HIPCHK(c, hipMalloc(&d_out, rcap * (u64)RW * 4));
    HIPCHK(c, hipMalloc(&d_cnt, 8));
    HIPCHK(c, hipMemcpy(d_in, packed.data(), packed.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(d_cnt, 0, 8));
    HIPCHK(c, launch(c->sh, 2, c->P, c->PT, c->B, (u64)n, 0, d_in, d_out, rcap, d_cnt, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    unsigned long long cnt = 0;
    HIPCHK(c, hipMemcpy(&cnt, d_cnt, 8, hipMemcpyDeviceToHost));
    const u64 got = std::min<u64>(cnt, rcap);
    std::vector<u32> recs(got * (u64)RW);
    if (got) HIPCHK(c, hipMemcpy(recs.data(), d_out, recs.size() * 4, hipMemcpyDeviceToHost));
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    (void)hipFree(d_cnt);
    // deterministic order: (parent, lane)
    std::vector<u64> order(got);
    for (u64 q = 0; q < got; ++q) order[q] = q;
    std::sort(order.begin(), order.end(), [&](u64 a, u64 b) {
        const u32* ra = &recs[a * RW];
        const u32* rb = &recs[b * RW];
        const u64 pa = (u64)ra[0] | ((u64)ra[1] << 32), pb = (u64)rb[0] | ((u64)rb[1] << 32);
        return pa != pb ? pa < pb : ra[2] < rb[2];
    });
    for (u64 q = 0; q < got && q < cap; ++q) {
        const u32* r = &recs[order[q] * RW];
        rmc_succ_view& s = out[q];
        memset(&s, 0, sizeof s);
        s.parent = (u64)r[0] | ((u64)r[1] << 32);
        s.instance = (int)r[2];
        s.family = family_of(c->P, (int)r[2]);
        s.in_constraint = (int)r[3];
        s.fingerprint = (u64)r[4] | ((u64)r[5] << 32);
        if (s.in_constraint) decode_state(c, r + 6, &s.state);
    }
    *n_out = (size_t)cnt;
    return 0;
}

}  // extern "C"
