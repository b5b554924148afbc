// rmc_wide.cpp — host side of the wide layout (raft_wide.h, rmc_wide.hip):
// the codec between rmc_state_view and the wide record, the BFS level loop,
// the counterexample walk, the successor listing and the random walks.  A
// ctx is wide when some bound of its config exceeds the packed capacity
// (rmc.h RMC_WIDE_MAX_*), e.g. the unbounded fields of MCraft.cfg as shipped
// under a depth bound, or Smokeraft's walks; RMC_FORCE_WIDE=1 forces it on a
// packed-size model (tests compare the two layouts on the same model).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rmc_ctx.h"

using namespace rmc;
using namespace rmc::wide;

namespace rmc_host {

bool wide_wanted(const rmc_config& g) {
    if (const char* e = getenv("RMC_FORCE_WIDE"))
        if (atoi(e)) return true;
    return g.max_term > RMC_MAX_TERM || g.max_log_len > RMC_MAX_LOG || g.max_msgs > RMC_MAX_MSGS ||
           g.max_dup > RMC_MAX_DUP;
}

int validate_wide(const rmc_config* c, std::string* why) {
    auto bad = [&](const char* s) { *why = s; return RMC_E_INVAL; };
    static_assert(wide::LW == RMC_WIDE_MAX_LOG && wide::KW == RMC_WIDE_MAX_MSGS && wide::TMAX == RMC_WIDE_MAX_TERM &&
                      wide::CMAX == RMC_WIDE_MAX_DUP && RMC_VIEW_LOG >= wide::LW && RMC_VIEW_MSGS >= wide::KW,
                  "the wide layout's capacity is rmc.h's RMC_WIDE_MAX_*");
    if (c->max_term < 1 || c->max_term > RMC_WIDE_MAX_TERM) return bad("max_term must be 1..255 (wide layout)");
    if (c->max_log_len < 0 || c->max_log_len > RMC_WIDE_MAX_LOG) return bad("max_log_len must be 0..32 (wide layout)");
    if (c->max_msgs < 0 || c->max_msgs > RMC_WIDE_MAX_MSGS) return bad("max_msgs must be 0..64 (wide layout)");
    if (c->max_dup < 1 || c->max_dup > RMC_WIDE_MAX_DUP) return bad("max_dup must be 1..255 (wide layout)");
    if (c->flags & (RMC_FLAG_SYMMETRY | RMC_FLAG_VERIFY_STATES | RMC_FLAG_SPILL))
        return bad("the wide layout (bounds beyond the packed capacity) supports no SYMMETRY, verification or spill");
    return 0;
}

void fill_wide_model(rmc_ctx* c) {
    const rmc_config& g = c->cfg;
    WModel& M = c->WM;
    M.S = g.n_servers;
    M.V = g.n_values;
    M.max_term = g.max_term;
    M.max_log = g.max_log_len;
    M.max_msgs = g.max_msgs;
    M.max_dup = g.max_dup;
    M.unbounded = (int)((g.flags >> 5) & 15u);
    M.bug_quorum = (g.flags & RMC_FLAG_BUG_QUORUM) ? 1 : 0;
    M.inv_mask = (int)g.invariants;
    M.L.init(M.S);
}

int wide_family(const rmc_ctx* c, int lane) { return lane == 255 ? -1 : c->WM.L.family(lane); }

// The BFS store's record (WideBufs.compact): the smallest that no state of the
// run can outgrow — each field either bounded by a CONSTRAINT within the record
// (a successor beyond it is out of the model anyway) or unbounded in a run of
// few enough levels.  2: the depth-sized WStateD (4 entries, 12 messages; after
// n steps a log holds at most n - 9 entries, n - 5 under the weakened quorum,
// and the bag at most n - 1 messages: raft_wide.h), 1: the compact WStateC (16,
// 16; one step adds at most one entry and one message), 0: the full WState.
// RMC_WIDE_COMPACT=0/1/2 overrides (A/B, tests).
static int wide_compact(const rmc_config& g) {
    if (const char* e = getenv("RMC_WIDE_COMPACT")) return std::max(0, std::min(2, atoi(e)));
    const int steps = g.max_depth > 0 ? g.max_depth - 1 : 1 << 30;
    const bool blog = (g.flags & RMC_FLAG_UNBOUNDED_LOG) == 0, bmsg = (g.flags & RMC_FLAG_UNBOUNDED_MSGS) == 0;
    const int lead = (g.flags & RMC_FLAG_BUG_QUORUM) ? 5 : 9;  // steps before a first log entry can exist
    if (((blog && g.max_log_len <= LWD) || steps - lead <= LWD) && ((bmsg && g.max_msgs <= KWD) || steps - 1 <= KWD))
        return 2;
    const bool logs = (blog && g.max_log_len <= LWC) || steps <= LWC;
    const bool msgs = (bmsg && g.max_msgs <= KWC) || steps <= KWC;
    return logs && msgs ? 1 : 0;
}
static size_t record_bytes(int kind) {
    return kind == 2 ? sizeof(WStateD) : kind == 1 ? sizeof(WStateC) : sizeof(WState);
}
size_t wide_record_bytes(const rmc_config& g) { return record_bytes(wide_compact(g)); }

// ---- codec ----------------------------------------------------------------------
int encode_wide(const rmc_ctx* c, const rmc_state_view& v, WState* out, std::string* why) {
    const int S = c->WM.S;
    auto bad = [&](const std::string& s) { *why = s; return RMC_E_INVAL; };
    WState& s = *out;
    wzero(&s, (int)sizeof s);
    if (v.n_servers != S) return bad("view n_servers differs from config");
    if (v.n_msgs < 0 || v.n_msgs > KW) return bad("too many messages for the wide bag");
    auto byte = [](int x, int lo, int hi) { return x >= lo && x <= hi; };
    for (int i = 0; i < S; ++i) {
        if (!byte(v.currentTerm[i], 0, TMAX)) return bad("currentTerm out of the wide range");
        if (!byte(v.state[i], 0, 2)) return bad("state out of range");
        if (v.votedFor[i] < -1 || v.votedFor[i] >= S) return bad("votedFor out of range");
        if (!byte(v.commitIndex[i], 0, 255)) return bad("commitIndex out of range");
        if (!byte(v.log_len[i], 0, LW)) return bad("log length out of the wide range");
        if ((v.votesResponded[i] | v.votesGranted[i]) >> S) return bad("vote set out of range");
        s.ct[i] = (uint8_t)v.currentTerm[i];
        s.st[i] = (uint8_t)v.state[i];
        s.vf[i] = v.votedFor[i] < 0 ? NIL : (uint8_t)v.votedFor[i];
        s.ci[i] = (uint8_t)v.commitIndex[i];
        s.len[i] = (uint8_t)v.log_len[i];
        s.vR[i] = (uint8_t)v.votesResponded[i];
        s.vG[i] = (uint8_t)v.votesGranted[i];
        for (int x = 0; x < v.log_len[i]; ++x) {
            if (!byte(v.log[i][x].term, 0, TMAX) || !byte(v.log[i][x].value, 0, 1)) return bad("log entry out of range");
            s.log[i][x].term = (uint8_t)v.log[i][x].term;
            s.log[i][x].value = (uint8_t)v.log[i][x].value;
        }
        for (int j = 0; j < S; ++j) {
            if (!byte(v.nextIndex[i][j], 1, 255) || !byte(v.matchIndex[i][j], 0, 255)) return bad("index out of range");
            s.ni[i][j] = (uint8_t)v.nextIndex[i][j];
            s.mi[i][j] = (uint8_t)v.matchIndex[i][j];
        }
    }
    for (int q = 0; q < v.n_msgs; ++q) {
        const rmc_msg_view& m = v.msgs[q];
        if (!byte(m.mtype, 0, 3)) return bad("mtype out of range");
        if (!byte(m.msource, 0, S - 1) || !byte(m.mdest, 0, S - 1)) return bad("message endpoint out of range");
        if (!byte(m.mterm, 0, TMAX)) return bad("mterm out of the wide range");
        if (!byte(m.count, 1, CMAX)) return bad("message count out of the wide range");
        WMsg w;
        wmsg_zero(w);
        w.type = (uint8_t)m.mtype;
        w.term = (uint8_t)m.mterm;
        w.src = (uint8_t)m.msource;
        w.dst = (uint8_t)m.mdest;
        switch (m.mtype) {
            case RVQ:
                if (!byte(m.mlastLogTerm, 0, TMAX) || !byte(m.mlastLogIndex, 0, 255))
                    return bad("RequestVoteRequest field out of range");
                w.b = (uint8_t)m.mlastLogTerm;
                w.c = (uint8_t)m.mlastLogIndex;
                break;
            case RVP:
                if (!byte(m.mlog_len, 0, LW)) return bad("mlog too long");
                w.a = (int8_t)(m.mvoteGranted != 0);
                w.n = (uint8_t)m.mlog_len;
                for (int x = 0; x < m.mlog_len; ++x) {
                    if (!byte(m.mlog[x].term, 0, TMAX) || !byte(m.mlog[x].value, 0, 1)) return bad("mlog entry out of range");
                    w.e[x].term = (uint8_t)m.mlog[x].term;
                    w.e[x].value = (uint8_t)m.mlog[x].value;
                }
                break;
            case AEQ:
                if (!byte(m.mprevLogIndex, -1, 127) || !byte(m.mprevLogTerm, 0, 255) || !byte(m.mentries_len, 0, 1) ||
                    !byte(m.mcommitIndex, 0, 255))
                    return bad("AppendEntriesRequest field out of range");
                w.a = (int8_t)m.mprevLogIndex;
                w.b = (uint8_t)m.mprevLogTerm;
                w.c = (uint8_t)m.mcommitIndex;
                w.n = (uint8_t)m.mentries_len;
                if (m.mentries_len) {
                    if (!byte(m.mentries[0].term, 0, TMAX) || !byte(m.mentries[0].value, 0, 1))
                        return bad("mentries entry out of range");
                    w.e[0].term = (uint8_t)m.mentries[0].term;
                    w.e[0].value = (uint8_t)m.mentries[0].value;
                }
                break;
            default:
                if (!byte(m.mmatchIndex, 0, 255)) return bad("mmatchIndex out of range");
                w.a = (int8_t)(m.msuccess != 0);
                w.b = (uint8_t)m.mmatchIndex;
        }
        for (int k = 0; k < s.nmsg; ++k)
            if (wmsg_cmp(s.msg[k], w) == 0) return bad("duplicate message in bag view");
        // insert sorted (the canonical order)
        int k = 0;
        while (k < s.nmsg && wmsg_cmp(s.msg[k], w) < 0) ++k;
        for (int r = s.nmsg; r > k; --r) {
            s.msg[r] = s.msg[r - 1];
            s.cnt[r] = s.cnt[r - 1];
        }
        s.msg[k] = w;
        s.cnt[k] = (uint8_t)m.count;
        s.nmsg += 1;
    }
    return 0;
}

template <class St>
void decode_wide(const rmc_ctx* c, const St& s, rmc_state_view* v) {
    const int S = c->WM.S;
    memset(v, 0, sizeof *v);
    v->n_servers = S;
    for (int i = 0; i < S; ++i) {
        v->currentTerm[i] = s.ct[i];
        v->state[i] = s.st[i];
        v->votedFor[i] = s.vf[i] == NIL ? -1 : s.vf[i];
        v->commitIndex[i] = s.ci[i];
        v->log_len[i] = s.len[i];
        for (int x = 0; x < s.len[i]; ++x) {
            v->log[i][x].term = s.log[i][x].term;
            v->log[i][x].value = s.log[i][x].value;
        }
        v->votesResponded[i] = s.vR[i];
        v->votesGranted[i] = s.vG[i];
        for (int j = 0; j < S; ++j) {
            v->nextIndex[i][j] = s.ni[i][j];
            v->matchIndex[i][j] = s.mi[i][j];
        }
    }
    v->n_msgs = s.nmsg;
    for (int q = 0; q < s.nmsg; ++q) {
        const auto& w = s.msg[q];
        rmc_msg_view& m = v->msgs[q];
        m.mtype = w.type;
        m.mterm = w.term;
        m.msource = w.src;
        m.mdest = w.dst;
        m.count = s.cnt[q];
        switch (w.type) {
            case RVQ: m.mlastLogTerm = w.b; m.mlastLogIndex = w.c; break;
            case RVP:
                m.mvoteGranted = w.a;
                m.mlog_len = w.n;
                for (int x = 0; x < w.n; ++x) { m.mlog[x].term = w.e[x].term; m.mlog[x].value = w.e[x].value; }
                break;
            case AEQ:
                m.mprevLogIndex = w.a;
                m.mprevLogTerm = w.b;
                m.mcommitIndex = w.c;
                m.mentries_len = w.n;
                if (w.n) { m.mentries[0].term = w.e[0].term; m.mentries[0].value = w.e[0].value; }
                break;
            default: m.msuccess = w.a; m.mmatchIndex = w.b;
        }
    }
}

// ---- context ----------------------------------------------------------------------
int create_wide(rmc_ctx* c) {
    fill_wide_model(c);
    const int compact = wide_compact(c->cfg);
    const u64 rec = record_bytes(compact);
    const u64 per_state = rec + 8 + 1;
    size_t fr = 0, tot = 0;
    (void)hipMemGetInfo(&fr, &tot);
    const u64 budget = (u64)((double)fr * 0.80);
    const u64 set_slots = set_slots_of(c->cfg.set_bytes);  // rmc_config.set_bytes (TLC -fpmem)
    u64 cap = c->cfg.state_capacity;
    if (set_slots && cap > set_slots / 2) {
        c->err = "state_capacity exceeds what a set of set_bytes " + std::to_string(c->cfg.set_bytes) + " holds";
        return RMC_E_INVAL;
    }
    if (cap == 0)
        cap = set_slots ? std::min<u64>(set_slots / 2, (budget - std::min<u64>(budget, set_slots * 8)) / per_state)
                        : budget / (per_state + 32);
    cap = std::max<u64>(std::min<u64>(cap, 1ull << 33), 1024);
    u64 slots = 1;
    while (slots < 2 * cap) slots <<= 1;
    if (set_slots) slots = std::max(slots, set_slots);
    c->table_slots = slots;
    WideBufs& B = c->WB;
    B = WideBufs{};
    B.cap = cap;
    B.tmask = slots - 1;
    B.compact = compact;
    if (hipMalloc(&B.store, cap * rec) != hipSuccess || hipMalloc(&B.parent, cap * 8) != hipSuccess ||
        hipMalloc(&B.act, cap) != hipSuccess || hipMalloc(&B.table, slots * 8) != hipSuccess ||
        hipMalloc(&B.ctr, sizeof(Counters)) != hipSuccess || hipMalloc(&c->w_staged, sizeof(WState)) != hipSuccess)
        return fail(c, RMC_E_NOMEM, "device allocation failed (wide layout, capacity " + std::to_string(cap) + " states)");
    c->B.ctr = B.ctr;  // reset_counters / read_counters work on it
    c->B.cap = cap;
    return 0;
}

void destroy_wide(rmc_ctx* c) {
    WideBufs& B = c->WB;
    (void)hipFree(B.store);
    (void)hipFree(B.parent);
    (void)hipFree(B.act);
    (void)hipFree(B.table);
    (void)hipFree(B.ctr);
    (void)hipFree(c->w_staged);
    B = WideBufs{};
    c->B.ctr = nullptr;
    c->w_staged = nullptr;
}

static u64 wide_salt(u64 seed) { return seed ? (mix64(seed) & ((1ull << 59) - 1)) : 0ull; }

// ---- BFS (TLC's worker loop on the wide layout) ----------------------------------------
int run_bfs_wide(rmc_ctx* c, rmc_progress_fn cb, void* user) {
    const auto t0 = std::chrono::steady_clock::now();
    auto secs = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    if (c->resume) return fail(c, RMC_E_STATE, "recover: not supported on the wide layout");
    WideBufs B = c->WB;
    B.salt = wide_salt(c->cfg.seed);
    c->have_target = 0;
    c->res = rmc_result{};
    c->res.set_slots = c->table_slots;
    c->level_start.clear();
    HIPCHK(c, launch_fill(B.table, c->table_slots * 8, 0, c->st));
    c->h_ctr->count = 0;
    if (int rc = reset_counters(c, false)) return rc;
    WState init;
    WStateC initc;
    WStateD initd;
    winit(c->WM, init);
    winit(c->WM, initc);
    winit(c->WM, initd);
    if (B.compact == 2) HIPCHK(c, hipMemcpyAsync(c->w_staged, &initd, sizeof initd, hipMemcpyHostToDevice, c->st));
    else if (B.compact) HIPCHK(c, hipMemcpyAsync(c->w_staged, &initc, sizeof initc, hipMemcpyHostToDevice, c->st));
    else HIPCHK(c, hipMemcpyAsync(c->w_staged, &init, sizeof init, hipMemcpyHostToDevice, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));  // (the staging copies live on this stack frame)
    HIPCHK(c, launch_wseed(c->WM, B, c->w_staged, 1, c->st));
    if (int rc = read_counters(c)) return rc;
    c->res.generated = 1;
    c->level_start.push_back(0);
    c->level_start.push_back(c->h_ctr->count);
    int depth = c->h_ctr->count ? 1 : 0;
    if (c->h_ctr->viol != ~0ull) {
        c->res.violated_inv = 1 << (int)(c->h_ctr->viol & 15);
        c->res.violation_depth = 1;
        c->have_target = 1;
        c->target_idx = c->h_ctr->viol >> 4;
    }
    const u64 CHUNK = 1ull << 22;
    while (!c->have_target) {
        const u64 lo = c->level_start[(size_t)depth - 1], hi = c->level_start[(size_t)depth];
        if (lo == hi) break;
        if (c->cfg.max_depth > 0 && depth >= c->cfg.max_depth) {
            c->res.left_on_queue = hi - lo;
            break;
        }
        if (int rc = reset_counters(c, true)) return rc;
        HIPCHK(c, hipEventRecord(c->ev0, c->st));
        for (u64 a = lo; a < hi; a += CHUNK) {
            HIPCHK(c, launch_wexpand(c->WM, B, a, std::min(hi, a + CHUNK), c->st));
            c->res.expand_launches += 1;
        }
        HIPCHK(c, hipEventRecord(c->ev1, c->st));
        if (int rc = read_counters(c)) return rc;
        float ms = 0.f;
        HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->res.expand_kernel_seconds += 1e-3 * ms;
        const Counters& k = *c->h_ctr;
        if (k.table_full) return fail(c, RMC_E_CAPACITY, "fingerprint set full");
        if (k.overflow >> 8) return fail(c, RMC_E_CAPACITY, capacity_message(c, k.overflow, depth));
        if (k.overflow)
            return fail(c, RMC_E_CAPACITY, "state store full (capacity " + std::to_string(B.cap) +
                                               " wide states); raise rmc_config.state_capacity");
        c->res.generated += k.generated;
        c->res.probes += k.probes;
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
    c->res.stored_here = c->res.distinct;
    const double Dd = (double)c->res.distinct, G = (double)c->res.generated;
    c->res.collision_probability = fp_collision_estimate(Dd, G, (c->WB.tmask + 1));
    c->res.seconds = secs();
    return 0;
}

int trace_wide(rmc_ctx* c, rmc_state_view* states, int32_t* families, int32_t* instances, size_t cap, size_t* len) {
    std::vector<u64> chain;
    std::vector<uint8_t> acts;
    u64 idx = c->target_idx;
    for (;;) {
        u64 p = 0;
        uint8_t a = 0;
        HIPCHK(c, hipMemcpy(&p, c->WB.parent + idx, 8, hipMemcpyDeviceToHost));
        HIPCHK(c, hipMemcpy(&a, c->WB.act + idx, 1, hipMemcpyDeviceToHost));
        chain.push_back(idx);
        acts.push_back(a);
        if (p == ~0ull || chain.size() > 100000) break;
        idx = p;
    }
    std::reverse(chain.begin(), chain.end());
    std::reverse(acts.begin(), acts.end());
    *len = chain.size();
    for (size_t q = 0; q < chain.size() && q < cap; ++q) {
        if (c->WB.compact == 2) {
            WStateD s;
            HIPCHK(c, hipMemcpy(&s, static_cast<const WStateD*>(c->WB.store) + chain[q], sizeof s, hipMemcpyDeviceToHost));
            if (states) decode_wide(c, s, &states[q]);
        } else if (c->WB.compact) {
            WStateC s;
            HIPCHK(c, hipMemcpy(&s, static_cast<const WStateC*>(c->WB.store) + chain[q], sizeof s, hipMemcpyDeviceToHost));
            if (states) decode_wide(c, s, &states[q]);
        } else {
            WState s;
            HIPCHK(c, hipMemcpy(&s, static_cast<const WState*>(c->WB.store) + chain[q], sizeof s, hipMemcpyDeviceToHost));
            if (states) decode_wide(c, s, &states[q]);
        }
        if (families) families[q] = wide_family(c, acts[q]);
        if (instances) instances[q] = acts[q] == 255 ? -1 : acts[q];
    }
    return 0;
}

int expand_wide(rmc_ctx* c, const rmc_state_view* states, size_t n, rmc_succ_view* out, size_t cap, size_t* n_out) {
    std::vector<WState> in(n);
    std::string why;
    for (size_t t = 0; t < n; ++t)
        if (encode_wide(c, states[t], &in[t], &why)) return fail(c, RMC_E_INVAL, "state " + std::to_string(t) + ": " + why);
    const u64 lanes = (u64)c->WM.L.off[10];
    const u64 rcap = std::max<u64>(1, std::min<u64>((u64)cap, n * lanes));
    WState* d_in = nullptr;
    WSucc* d_out = nullptr;
    unsigned long long* d_cnt = nullptr;
    HIPCHK(c, hipMalloc(&d_in, n * sizeof(WState)));
    HIPCHK(c, hipMalloc(&d_out, rcap * sizeof(WSucc)));
    HIPCHK(c, hipMalloc(&d_cnt, 8));
    HIPCHK(c, hipMemcpy(d_in, in.data(), n * sizeof(WState), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(d_cnt, 0, 8));
    HIPCHK(c, launch_wlist(c->WM, d_in, (u64)n, d_out, rcap, d_cnt, wide_salt(c->cfg.seed), c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    unsigned long long cnt = 0;
    HIPCHK(c, hipMemcpy(&cnt, d_cnt, 8, hipMemcpyDeviceToHost));
    const u64 got = std::min<u64>(cnt, rcap);
    std::vector<WSucc> recs(got);
    if (got) HIPCHK(c, hipMemcpy(recs.data(), d_out, got * sizeof(WSucc), hipMemcpyDeviceToHost));
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    (void)hipFree(d_cnt);
    std::sort(recs.begin(), recs.end(), [](const WSucc& a, const WSucc& b) {
        return a.parent != b.parent ? a.parent < b.parent : a.lane < b.lane;
    });
    for (u64 q = 0; q < got && q < cap; ++q) {
        rmc_succ_view& s = out[q];
        memset(&s, 0, sizeof s);
        s.parent = recs[q].parent;
        s.instance = recs[q].lane;
        s.family = wide_family(c, recs[q].lane);
        s.in_constraint = recs[q].in_model;
        s.fingerprint = recs[q].fp;
        if (s.in_constraint) decode_wide(c, recs[q].state, &s.state);
    }
    *n_out = (size_t)cnt;
    return 0;
}

int smoke_views(const rmc_ctx* c, const rmc_sim_config& sc, std::vector<rmc_state_view>* views, std::string* why);

int sim_wide(rmc_ctx* c, const rmc_sim_config* sc, rmc_sim_result* out, i64 rec_beh, std::vector<rmc_state_view>* rec) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<WState> inits;
    std::string why;
    if (sc->smoke_k > 0) {
        std::vector<rmc_state_view> views;
        if (int rc = smoke_views(c, *sc, &views, &why)) return fail(c, rc, why);
        inits.resize(views.size());
        for (size_t q = 0; q < views.size(); ++q)
            if (int rc = encode_wide(c, views[q], &inits[q], &why)) return fail(c, rc, why);
    } else {
        inits.resize(1);
        winit(c->WM, inits[0]);
    }
    const u64 n_init = inits.size();
    WState *d_init = nullptr, *d_rec = nullptr;
    SimCounters* d_out = nullptr;
    HIPCHK(c, hipMalloc(&d_init, n_init * sizeof(WState)));
    HIPCHK(c, hipMalloc(&d_out, sizeof(SimCounters)));
    if (rec) HIPCHK(c, hipMalloc(&d_rec, (size_t)sc->depth * sizeof(WState)));
    SimCounters h{};
    h.viol = ~0ull;
    HIPCHK(c, hipMemcpy(d_init, inits.data(), n_init * sizeof(WState), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(d_out, &h, sizeof h, hipMemcpyHostToDevice));
    HIPCHK(c, hipEventRecord(c->ev0, c->st));
    HIPCHK(c, launch_wsimulate(c->WM, d_init, n_init, sc->behaviours, sc->depth, sc->seed, sc->mode, d_out, rec_beh,
                               d_rec, c->st));
    HIPCHK(c, hipEventRecord(c->ev1, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    HIPCHK(c, hipMemcpy(&h, d_out, sizeof h, hipMemcpyDeviceToHost));
    if (rec) {
        std::vector<WState> ws((size_t)(h.steps + 1));
        HIPCHK(c, hipMemcpy(ws.data(), d_rec, ws.size() * sizeof(WState), hipMemcpyDeviceToHost));
        rec->resize(ws.size());
        for (size_t q = 0; q < ws.size(); ++q) decode_wide(c, ws[q], &(*rec)[q]);
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

}  // namespace rmc_host
