// rmc_dist.cpp — sharded BFS over several GPUs behind the C ABI (rmc_shard).
//
// One ctx per GPU, each a rank of a state-space partition (SURVEY.md §8e;
// replaces TLC's distributed mode).  Per BFS level every rank expands the
// frontier it owns in ROUNDS; a round's exchange is two-phase, fingerprint
// first:
//   phase 1  k_expand<DIST> puts the key of every successor owned elsewhere
//            (and not in the sent-cache) in that owner's key outbox with a
//            local ticket (parent, lane); a count all-to-all tells every rank
//            what it receives; keys all-to-all; the owner inserts them
//            (k_owner_insert), answers new/seen with 1 byte per key and
//            counts per source the states it will receive; replies
//            all-to-all (the reverse of the key exchange);
//   phase 2  k_materialize_remote re-derives the accepted successors from
//            their tickets into per-owner state outboxes (counting them);
//            states all-to-all; the owner stores them (k_store_remote).
// Pipelining: two outbox sets.  The ctx stream expands round k + 1 into one
// set while the exchange stream (xs) runs round k's exchange on the other, so
// the host's two count read-backs per round wait while the GPU expands.  A
// level ends with one all-gather of the device counters.  Keys that do not
// fit an outbox are parked (B.ovf) and sent in later rounds of the same level:
// an outbox overflow costs a round, never the run.
// Collectives run on RCCL over xGMI (one communicator per ctx) or on a
// caller-supplied host transport (gloo in the tests, where several ranks share
// one GPU; every collective is then a synchronous host round trip).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "rmc_ctx.h"

using namespace rmc;
using namespace rmc_host;

namespace {

// Bytes per phase-1 key record: the raw fingerprint (k, s32) as three u32
// {k lo, k hi, s32} (raft_packed.h Fp, put_key; the owner derives its own
// table value and slot).
constexpr u64 KEYB = 12;

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- deadlines ---------------------------------------------------------------------
// Every wait of the sharded loop on other ranks has a deadline
// (RMC_DIST_TIMEOUT_S, default 300 s): a collective that has not completed in
// time aborts the RCCL communicator (ncclCommAbort also ends the kernels
// waiting inside it) and fails the call on this rank, naming the level, the
// round and the phase, instead of hanging until an outer time limit.  The
// communicator is non-blocking (ncclConfig_t.blocking = 0), so connection
// set-up inside a group call is polled under the same deadline.  A host
// transport applies its own deadline inside its callbacks (rmc.h).
std::string where(const rmc_ctx* c) {
    const DistState& D = c->dist;
    return "rank " + std::to_string(D.rank) + " of " + std::to_string(D.world) + ", level " +
           std::to_string(D.lvl) + ", round " + std::to_string(D.rnd) + ", phase " + D.phase;
}

// ncclCommAbort of a communicator whose peers never connected can itself wait
// on them (the bootstrap of an unfinished init): it runs on a helper thread,
// waited for at most kAbortWait s; past that the call returns and the helper
// is left to the process exit (after a deadline the caller ends the process,
// rmc.h).  Returns whether the abort completed.
constexpr double kAbortWait = 10.0;
bool abort_bounded(ncclComm_t comm) {
    auto done = std::make_shared<std::atomic<int>>(0);
    std::thread([comm, done] {
        (void)ncclCommAbort(comm);
        done->store(1);
    }).detach();
    const double t0 = now_s();
    while (!done->load() && now_s() - t0 < kAbortWait) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    return done->load() != 0;
}

// pending: the caller left a communicator it could not abort (communicator init).
int deadline_fail(rmc_ctx* c, const char* what, int pending = 0) {
    DistState& D = c->dist;
    D.aborted = 1;
    bool aborted = !pending;
    if (D.rccl && D.comm) {
        aborted = abort_bounded(D.comm);
        D.comm = nullptr;
    }
    if (D.rccl) D.abort_pending = aborted ? 0 : 1;
    char t[32];
    snprintf(t, sizeof t, "%g", D.timeout_s);
    return fail(c, RMC_E_HIP, std::string("sharded search: ") + what + " did not complete within the " + t +
                                  " s deadline (RMC_DIST_TIMEOUT_S) at " + where(c) +
                                  (!D.rccl ? "" : aborted ? "; the RCCL communicator was aborted"
                                                          : "; the RCCL communicator's abort is still pending "
                                                            "(end the process)"));
}

// Wait for an event of the exchange path under the deadline: spin first (a
// round's read-back is on the critical path), then back off.
int xwait(rmc_ctx* c, hipEvent_t ev) {
    DistState& D = c->dist;
    const double t0 = now_s();
    for (u64 spin = 0;; ++spin) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady)
            return fail(c, RMC_E_HIP, std::string("hipEventQuery: ") + hipGetErrorString(e) + " at " + where(c));
        if ((spin & 63) == 0) {
            const double dt = now_s() - t0;
            if (dt > D.timeout_s) return deadline_fail(c, "a wait on the exchange");
            // a level's expansion takes up to tens of ms: poll without sleeping for
            // the first 100 ms (a 20-us sleep wakes 50-80 us late, once per wait),
            // then gently (a stalled peer)
            if (dt > 0.1) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    D.wait_seconds += now_s() - t0;
    return 0;
}

// The result of an RCCL call on the non-blocking communicator: ncclInProgress
// is polled (ncclCommGetAsyncError) until the call is enqueued, under the deadline.
int nccl_done(rmc_ctx* c, ncclResult_t r, const char* what) {
    DistState& D = c->dist;
    if (r == ncclInProgress || (r == ncclSuccess && D.nonblocking)) {
        const double t0 = now_s();
        for (u64 spin = 0;; ++spin) {
            if (!D.comm) return fail(c, RMC_E_HIP, std::string(what) + ": no communicator at " + where(c));
            if (ncclCommGetAsyncError(D.comm, &r) != ncclSuccess) break;
            if (r != ncclInProgress) break;
            if ((spin & 63) == 0 && now_s() - t0 > D.timeout_s) return deadline_fail(c, what);
            if (spin > 4096) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    if (r != ncclSuccess) return fail(c, RMC_E_HIP, std::string(what) + ": " + ncclGetErrorString(r) + " at " + where(c));
    return 0;
}

#define NCCLCHK(c, expr)                                              \
    do {                                                              \
        if (int rc_ = nccl_done((c), (expr), #expr)) return rc_;      \
    } while (0)

// The host transport's callbacks return non-zero on failure, their own
// deadline included (rmc.h): the call fails naming where; a callback that
// failed after the deadline had passed is reported as the deadline.
int host_fail(rmc_ctx* c, const char* what, double t0) {
    const DistState& D = c->dist;
    if (now_s() - t0 >= 0.9 * D.timeout_s) {
        char t[32];
        snprintf(t, sizeof t, "%g", D.timeout_s);
        return fail(c, RMC_E_HIP, std::string("sharded search: the host transport's ") + what +
                                      " did not complete within the " + t + " s deadline (RMC_DIST_TIMEOUT_S) at " +
                                      where(c));
    }
    return fail(c, RMC_E_HIP, std::string("host transport ") + what + " failed at " + where(c));
}

// All-to-all of per-peer byte blocks living on the device, on the exchange
// stream: block p of the send side is sbuf + soff[p] (scnt[p] bytes) for rank
// p; block p of the receive side lands at rbuf + roff[p] (rcnt[p] bytes) from
// rank p.
int a2a(rmc_ctx* c, const void* sbuf, const u64* soff, const u64* scnt, void* rbuf, const u64* roff, const u64* rcnt) {
    DistState& D = c->dist;
    const int W = D.world;
    if (D.rccl) {
        bool any = false;
        for (int p = 0; p < W; ++p) any |= scnt[p] || rcnt[p];
        if (!any) return 0;
        NCCLCHK(c, ncclGroupStart());
        for (int p = 0; p < W; ++p) {
            if (scnt[p]) {
                const ncclResult_t r = ncclSend((const char*)sbuf + soff[p], scnt[p], ncclUint8, p, D.comm, D.xs);
                if (r != ncclSuccess && r != ncclInProgress) {
                    (void)ncclGroupEnd();
                    return nccl_done(c, r, "ncclSend");
                }
            }
            if (rcnt[p]) {
                const ncclResult_t r = ncclRecv((char*)rbuf + roff[p], rcnt[p], ncclUint8, p, D.comm, D.xs);
                if (r != ncclSuccess && r != ncclInProgress) {
                    (void)ncclGroupEnd();
                    return nccl_done(c, r, "ncclRecv");
                }
            }
        }
        NCCLCHK(c, ncclGroupEnd());
        return 0;
    }
    u64 st = 0, rt = 0;
    for (int p = 0; p < W; ++p) { st += scnt[p]; rt += rcnt[p]; }
    D.stage_send.resize(std::max<u64>(st, 1));
    D.stage_recv.resize(std::max<u64>(rt, 1));
    u64 o = 0;
    for (int p = 0; p < W; ++p) {
        if (scnt[p])
            HIPCHK(c, hipMemcpyAsync(D.stage_send.data() + o, (const char*)sbuf + soff[p], scnt[p], hipMemcpyDeviceToHost,
                                     D.xs));
        o += scnt[p];
    }
    HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
    if (int rc = xwait(c, D.ev_h)) return rc;
    const double th = now_s();
    if (D.host.alltoallv(D.host.user, D.stage_send.data(), scnt, D.stage_recv.data(), rcnt))
        return host_fail(c, "alltoallv", th);
    o = 0;
    for (int p = 0; p < W; ++p) {
        if (rcnt[p])
            HIPCHK(c, hipMemcpyAsync((char*)rbuf + roff[p], D.stage_recv.data() + o, rcnt[p], hipMemcpyHostToDevice, D.xs));
        o += rcnt[p];
    }
    HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
    return xwait(c, D.ev_h);
}

// All-to-all of `per` u64 per peer between device buffers (the count rows).
int a2a_u64(rmc_ctx* c, const u64* send, u64* recv, u64 per) {
    DistState& D = c->dist;
    if (D.world == 1) {  // a world of one: the row to itself, no collective
        HIPCHK(c, hipMemcpyAsync(recv, send, per * 8, hipMemcpyDeviceToDevice, D.xs));
        return 0;
    }
    if (D.rccl) {
        NCCLCHK(c, ncclAllToAll(send, recv, per, ncclUint64, D.comm, D.xs));
        return 0;
    }
    std::vector<u64> off((size_t)D.world), cnt((size_t)D.world, per * 8);
    for (int p = 0; p < D.world; ++p) off[(size_t)p] = (u64)p * per * 8;
    return a2a(c, send, off.data(), cnt.data(), recv, off.data(), cnt.data());
}

// All-gather of `bytes` host bytes per rank into all (world * bytes, rank order).
int allgather(rmc_ctx* c, const void* mine, u64 bytes, void* all) {
    DistState& D = c->dist;
    if (!D.rccl) {
        const double th = now_s();
        if (D.host.allgather(D.host.user, mine, bytes, all)) return host_fail(c, "allgather", th);
        return 0;
    }
    const bool big = bytes > D.ag_cap;  // rows are small: the staging buffer is allocated once
    void* d_buf = D.ag_dev;
    if (big) HIPCHK(c, hipMallocAsync(&d_buf, bytes * (u64)(D.world + 1), D.xs));
    char* d_in = (char*)d_buf + bytes * (u64)D.world;
    HIPCHK(c, hipMemcpyAsync(d_in, mine, bytes, hipMemcpyHostToDevice, D.xs));
    NCCLCHK(c, ncclAllGather(d_in, d_buf, bytes, ncclUint8, D.comm, D.xs));
    HIPCHK(c, hipMemcpyAsync(all, d_buf, bytes * (u64)D.world, hipMemcpyDeviceToHost, D.xs));
    if (big) HIPCHK(c, hipFreeAsync(d_buf, D.xs));
    HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
    return xwait(c, D.ev_h);
}

// All-gather of this rank's device counters (the level statistics), after
// every kernel of the level on both streams.
int allgather_counters(rmc_ctx* c, Counters* rows) {
    DistState& D = c->dist;
    HIPCHK(c, hipEventRecord(D.ev_c, c->st));
    HIPCHK(c, hipStreamWaitEvent(D.xs, D.ev_c, 0));
    const u64 bytes = sizeof(Counters);
    if (D.rccl) {
        NCCLCHK(c, ncclAllGather(c->B.ctr, D.ag_dev, bytes, ncclUint8, D.comm, D.xs));
        HIPCHK(c, hipMemcpyAsync(rows, D.ag_dev, bytes * (u64)D.world, hipMemcpyDeviceToHost, D.xs));
        HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
        return xwait(c, D.ev_h);
    }
    Counters mine;
    HIPCHK(c, hipMemcpyAsync(&mine, c->B.ctr, bytes, hipMemcpyDeviceToHost, D.xs));
    HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
    if (int rc = xwait(c, D.ev_h)) return rc;
    const double th = now_s();
    if (D.host.allgather(D.host.user, &mine, bytes, rows)) return host_fail(c, "allgather", th);
    return 0;
}

// Replicated level: every rank's records (n[p] of them, rb bytes each) into
// D.rep_buf, contiguous in rank order; this rank's own block is copied locally.
int gather_level(rmc_ctx* c, const std::vector<u64>& n, u64 rb) {
    DistState& D = c->dist;
    const int W = D.world, me = D.rank;
    std::vector<u64> off((size_t)W + 1, 0);
    for (int p = 0; p < W; ++p) off[(size_t)p + 1] = off[(size_t)p] + n[(size_t)p];
    char* dst = (char*)D.rep_buf;
    if (n[(size_t)me])
        HIPCHK(c, hipMemcpyAsync(dst + off[(size_t)me] * rb, D.rep_send, n[(size_t)me] * rb, hipMemcpyDeviceToDevice,
                                 D.xs));
    if (W == 1) return 0;
    if (D.rccl) {
        bool any = false;
        for (int p = 0; p < W; ++p) any |= p != me && (n[(size_t)p] || n[(size_t)me]);
        if (!any) return 0;
        NCCLCHK(c, ncclGroupStart());
        for (int p = 0; p < W; ++p) {
            if (p == me) continue;
            ncclResult_t r = ncclSuccess;
            if (n[(size_t)me]) r = ncclSend(D.rep_send, n[(size_t)me] * rb, ncclUint8, p, D.comm, D.xs);
            if ((r == ncclSuccess || r == ncclInProgress) && n[(size_t)p])
                r = ncclRecv(dst + off[(size_t)p] * rb, n[(size_t)p] * rb, ncclUint8, p, D.comm, D.xs);
            if (r != ncclSuccess && r != ncclInProgress) {
                (void)ncclGroupEnd();
                return nccl_done(c, r, "ncclSend/ncclRecv (level all-gather)");
            }
        }
        NCCLCHK(c, ncclGroupEnd());
        return 0;
    }
    // host transport: this rank's block to every peer (the block repeated per destination)
    const u64 mine = n[(size_t)me] * rb;
    std::vector<u64> scnt((size_t)W), rcnt((size_t)W);
    for (int p = 0; p < W; ++p) {
        scnt[(size_t)p] = p == me ? 0 : mine;
        rcnt[(size_t)p] = p == me ? 0 : n[(size_t)p] * rb;
    }
    D.stage_send.resize(std::max<u64>(mine * (u64)(W - 1), 1));
    D.stage_recv.resize(std::max<u64>((off[(size_t)W] - n[(size_t)me]) * rb, 1));
    if (mine) HIPCHK(c, hipMemcpyAsync(D.stage_send.data(), D.rep_send, mine, hipMemcpyDeviceToHost, D.xs));
    HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
    if (int rc = xwait(c, D.ev_h)) return rc;
    for (int q = 1; q < W - 1; ++q) memcpy(D.stage_send.data() + (u64)q * mine, D.stage_send.data(), mine);
    const double th = now_s();
    if (D.host.alltoallv(D.host.user, D.stage_send.data(), scnt.data(), D.stage_recv.data(), rcnt.data()))
        return host_fail(c, "alltoallv (level all-gather)", th);
    u64 o = 0;
    for (int p = 0; p < W; ++p) {
        if (rcnt[(size_t)p])
            HIPCHK(c, hipMemcpyAsync(dst + off[(size_t)p] * rb, D.stage_recv.data() + o, rcnt[(size_t)p],
                                     hipMemcpyHostToDevice, D.xs));
        o += rcnt[(size_t)p];
    }
    HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
    return xwait(c, D.ev_h);
}

float elapsed_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

}  // namespace

namespace rmc_host {

void free_dist(rmc_ctx* c) {
    DistState& D = c->dist;
    if (D.abort_pending) {  // RCCL kernels may still wait on these buffers: leave them to the process exit
        D = DistState{};
        D.aborted = 1;
        D.abort_pending = 1;
        return;
    }
    if (D.xs) (void)hipStreamSynchronize(D.xs);
    (void)hipFree(c->B.sent);
    (void)hipFree(c->B.ovf);
    for (auto& S : D.set) {
        (void)hipFree(S.key_out);
        (void)hipFree(S.tick_out);
        (void)hipFree(S.ocount);
        (void)hipFree(S.pool);
        (void)hipFree(S.cx);
        if (S.h_cx) (void)hipHostFree(S.h_cx);
        for (hipEvent_t* e : {&S.ev_exp, &S.ev_free, &S.k0, &S.k1, &S.x0, &S.x1})
            if (*e) (void)hipEventDestroy(*e);
        S = DistState::Set{};
    }
    for (hipEvent_t* e : {&D.ev_cnt, &D.ev_acc, &D.ev_c, &D.ev_x, &D.ev_h})
        if (*e) { (void)hipEventDestroy(*e); *e = nullptr; }
    (void)hipFree(D.rep_send);
    (void)hipFree(D.rep_buf);
    D.rep_send = nullptr;
    D.rep_buf = nullptr;
    (void)hipFree(D.key_in);
    (void)hipFree(D.rep_out);
    (void)hipFree(D.rep_in);
    (void)hipFree(D.st_in);
    (void)hipFree(c->B.st_out);
    (void)hipFree(D.sa);
    if (D.h_sa) (void)hipHostFree(D.h_sa);
    (void)hipFree(D.ag_dev);
    if (D.comm) {  // finalize (polled and bounded on a non-blocking communicator), then destroy
        ncclResult_t r = ncclCommFinalize(D.comm);
        const double t0 = now_s();
        while (r == ncclInProgress && now_s() - t0 < 10.0) {
            if (ncclCommGetAsyncError(D.comm, &r) != ncclSuccess) break;
            if (r == ncclInProgress) std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        if (r == ncclSuccess) (void)ncclCommDestroy(D.comm);
        else (void)ncclCommAbort(D.comm);
    }
    if (D.xs) (void)hipStreamDestroy(D.xs);
    c->B.sent = nullptr; c->B.key_out = nullptr; c->B.tick_out = nullptr; c->B.ocount = nullptr;
    c->B.st_out = nullptr; c->B.scount = nullptr; c->B.ovf = nullptr; c->B.ovf_cap = 0;
    D.key_in = nullptr; D.rep_out = nullptr; D.rep_in = nullptr; D.st_in = nullptr; D.sa = nullptr; D.h_sa = nullptr;
    D.ag_dev = nullptr;
    D.ag_cap = 0;
    D.comm = nullptr;
    D.xs = nullptr;
    D.on = 0;
    D.aborted = 0;
}

int run_bfs_sharded(rmc_ctx* c, rmc_progress_fn cb, void* user) {
    DistState& D = c->dist;
    const int W = D.world, me = D.rank;
    const u64 RB = (u64)(c->NW + 4) * 4;  // state record: packed state, global parent ref, footprint
    const u64 RBR = (u64)(c->NW + 6) * 4;  // replicated-level record (RepRec)
    const u64 kcap = c->B.kcap;
    const double t0 = now_s();
    if (D.aborted) return fail(c, RMC_E_STATE, "sharded search: the communicator was aborted by an earlier deadline");
    D.lvl = 0;
    D.rnd = 0;
    D.phase = "start";
    // rmc_recover restored this rank's levels, parents and set (every rank of
    // the checkpoint's world, each from its own part)
    const bool resume = c->resume != 0;
    c->resume = 0;
    const rmc_result saved = c->res;
    c->res = rmc_result{};
    c->res.set_slots = c->table_slots;
    if (!resume) c->level_start.clear();
    c->have_target = 0;
    D.keys_sent = D.states_sent = D.chunks = D.parked = 0;
    D.xfer_seconds = D.wait_seconds = 0;
    D.rep_levels = 0;
    // Set epochs as on one GPU (rmc_run_bfs, raft_packed.h c_set_ep): a run after
    // the ctx's first takes the next epoch instead of clearing the set.  The
    // send-marker kernels re-derive every remote key from its materialised
    // successor, never from a set value; SYMMETRY and verification (the lossy
    // sent-cache kernel recovers raw keys from set values) keep an untagged set.
    const char* epe = getenv("RMC_SET_EPOCH");
    const u32 ep_max = epe ? (u32)std::min(255, std::max(0, atoi(epe))) : 255u;
    const bool tagged = ep_max > 0 && !c->sh.verify && !c->sh.sym;
    if (!resume) {
        if (tagged && c->set_epoch >= 1 && c->set_epoch < ep_max) {
            c->set_epoch += 1;
        } else {
            HIPCHK(c, launch_fill(c->B.table, c->table_slots * 8, 0, c->st));
            c->set_epoch = tagged ? 1 : 0;
        }
    }
    if (c->B.sent) HIPCHK(c, launch_fill(c->B.sent, D.sent_slots * 8, 0, c->st));
    const bool verify = c->sh.verify;
    if (verify && !resume) HIPCHK(c, launch_fill(c->B.sidx, c->table_slots * 8, 0xFF, c->st));
    HIPCHK(c, set_fp_salt(c->sh, c->cfg.seed, c->set_epoch, c->st));
    if (resume) c->h_ctr->count = c->level_start.back();
    if (int rc = reset_counters(c, resume)) return rc;
    // ---- Init (raft.tla:125-129): stored by its owner only
    if (!resume) {
        rmc_state_view iv;
        init_view(c->cfg, &iv);
        std::vector<u32> packed((size_t)c->NW);
        std::string why;
        if (encode_view(c, iv, packed.data(), &why)) return fail(c, RMC_E_INVAL, why);
        HIPCHK(c, hipMemcpyAsync(c->d_staged, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, c->st));
        HIPCHK(c, launch(c->sh, 1, c->P, c->PT, c->B, 1, 0, c->d_staged, nullptr, 0, nullptr, c->st));
    }
    std::vector<Counters> rows((size_t)W);
    // level end: the all-gathered device counters; errors stop every rank alike
    bool rows_final = false;  // the level's last count row carried every rank's final counters
    auto level_end = [&]() -> int {
        D.phase = "level end (counter all-gather)";
        if (!rows_final) {
            if (int rc = allgather_counters(c, rows.data())) return rc;
        }
        rows_final = false;
        *c->h_ctr = rows[(size_t)me];
        for (int r = 0; r < W; ++r) {
            const Counters& k = rows[(size_t)r];
            if (k.table_full) return fail(c, RMC_E_CAPACITY, "fingerprint set full on rank " + std::to_string(r));
            if (k.overflow >> 8) return fail(c, RMC_E_CAPACITY, capacity_message(c, k.overflow, D.lvl));
            if (k.overflow & 4u) return fail(c, RMC_E_CAPACITY, "verification buffer full on rank " + std::to_string(r));
            if (k.overflow & 8u)
                return fail(c, RMC_E_HIP, "verification: a fingerprint without a published state on rank " +
                                              std::to_string(r));
            if (k.overflow & 2u)
                return fail(c, RMC_E_CAPACITY, "exchange parking buffer full on rank " + std::to_string(r) +
                                                   " (raise keys_per_dest)");
            if (k.overflow)
                return fail(c, RMC_E_CAPACITY, "state store full on rank " + std::to_string(r) +
                                                   " (raise rmc_config.state_capacity)");
        }
        return 0;
    };
    if (int rc = level_end()) return rc;
    if (!resume) {
        c->level_start.push_back(0);
        c->level_start.push_back(c->h_ctr->count);
    }
    if (verify && !resume && c->h_ctr->count)  // slot -> store index of the initial state(s)
        HIPCHK(c, launch(c->sh, 5, c->P, c->PT, c->B, 0, c->h_ctr->count, nullptr, nullptr, 0, nullptr, c->st));
    u64 total_prev = 0;
    std::vector<u64> count_before((size_t)W);  // every rank's store count when the current level began
    for (int r = 0; r < W; ++r) {
        total_prev += rows[(size_t)r].count;
        count_before[(size_t)r] = rows[(size_t)r].count;
    }
    if (resume && total_prev != saved.distinct)
        return fail(c, RMC_E_IO, "recover: the ranks' parts hold " + std::to_string(total_prev) +
                                     " states, the checkpoint " + std::to_string(saved.distinct));
    for (int r = 0; r < W && !c->have_target && !resume; ++r)  // Init's violation check (level 1)
        if (rows[(size_t)r].viol != ~0ull) {
            c->res.violated_inv = 1 << (int)(rows[(size_t)r].viol & 15);
            c->res.violation_depth = 1;
            c->have_target = 1;
            c->target_idx = ((u64)r << 48) | (rows[(size_t)r].viol >> 4);
        }
    // every rank's frontier size (replicated levels need them all), and
    // whether some rank passed a progress callback (the per-level stop vote
    // runs only then)
    std::vector<u64> fsz((size_t)W);
    int any_cb = 0;
    {
        D.phase = "start (frontier sizes)";
        const u64 mine[2] = {c->level_start.back() - c->level_start[c->level_start.size() - 2], cb ? 1ull : 0ull};
        std::vector<u64> all(2 * (size_t)W);
        if (int rc = allgather(c, mine, sizeof mine, all.data())) return rc;
        for (int r = 0; r < W; ++r) {
            fsz[(size_t)r] = all[2 * (size_t)r];
            any_cb |= all[2 * (size_t)r + 1] ? 1 : 0;
        }
    }
    u64 generated = resume ? saved.generated : 1, probes = resume ? saved.probes : 0;
    int depth = resume ? c->resume_depth : 1;
    // Replicated levels: the plain kernel (every shape), models with a
    // CONSTRAINT on every field (the capacity pass reads the store)
    // (a world of one has nothing to gather: its levels run as plain rounds)
    const bool rep_ok = W > 1 && !verify && !c->sh.sym && !c->P.unbounded && D.rep_max > 0;
    // Round sizing: rho = most keys one round sends one owner, per expanded
    // state, from the previous rounds (it varies along a frontier: states
    // received from other ranks are appended after the local ones).  A round
    // aims at an outbox half full; what does not fit is parked, not lost.
    double rho = 1.0;
    u64 vpub = c->h_ctr->count;  // verification: states [0, vpub) are published (slot -> index)
    // cx: [W] sent blocks of kRowWords, [1] novf, [W] received blocks (count, flags, counters)
    const u64 RWD = (u64)kRowWords;
    const u64 row_len = 2 * RWD * (u64)W + 1;
    auto rx = [&](const u64* cx, int p) { return cx + RWD * (u64)W + 1 + RWD * (u64)p; };  // block from p
    while (!c->have_target) {
        const u64 lo = c->level_start[(size_t)depth - 1], hi = c->level_start[(size_t)depth];
        D.lvl = depth;
        D.rnd = 0;
        if (c->cfg.max_depth > 0 && depth >= c->cfg.max_depth) {
            c->res.left_on_queue = 0;
            for (u64 x : fsz) c->res.left_on_queue += x;
            break;
        }
        if (D.stall_rank == me && D.stall_level == depth) {  // test hook: this rank stops answering
            fprintf(stderr, "[rmc rank %d] RMC_DIST_STALL_RANK: stalling %.1f s at level %d\n", me, D.stall_s, depth);
            std::this_thread::sleep_for(std::chrono::duration<double>(D.stall_s));
        }
        if (int rc = reset_counters(c, true)) return rc;
        bool rep_timed = false;
        u64 ftot = 0;
        for (u64 x : fsz) ftot += x;
        if (rep_ok && ftot <= D.rep_max) {
            // ---- a replicated level: every rank gathers the whole frontier,
            // expands all of it and keeps the successors it owns; no key or
            // state exchange, one all-gather of the level's records
            D.phase = "replicated level (frontier all-gather)";
            if (hi > lo) HIPCHK(c, launch(c->sh, 13, c->P, c->PT, c->B, lo, hi, nullptr, D.rep_send, 0, nullptr, c->st));
            HIPCHK(c, hipEventRecord(D.ev_c, c->st));
            HIPCHK(c, hipStreamWaitEvent(D.xs, D.ev_c, 0));
            if (int rc = gather_level(c, fsz, RBR)) return rc;
            HIPCHK(c, hipEventRecord(D.ev_x, D.xs));
            HIPCHK(c, hipStreamWaitEvent(c->st, D.ev_x, 0));
            D.phase = "replicated level (expansion)";
            DevBufs Bb = c->B;
            Bb.rep = D.rep_buf;
            // one launch (rep_max <= 2^24 records); timed by events read after the level end
            HIPCHK(c, hipEventRecord(D.set[0].k0, c->st));
            HIPCHK(c, launch(c->sh, 12, c->P, c->PT, Bb, 0, ftot, nullptr, nullptr, 0, nullptr, c->st));
            HIPCHK(c, hipEventRecord(D.set[0].k1, c->st));
            rep_timed = ftot != 0;
            c->res.expand_launches += 1;
            D.rep_levels += 1;
            D.chunks += 1;
        } else {
        u64 cursor = lo, ovf_known = 0, ovf_done = 0;
        const u64 frontier = hi - lo;
        // at least D.split rounds for a large level, so one round's count
        // exchange and read-back overlap the next round's expansion
        const u64 split_cap = frontier >= (1ull << 21) ? (frontier + D.split - 1) / (u64)D.split : frontier;
        u64 round_states[2] = {0, 0};  // states expanded by the round held in each set
        int round_kind[2] = {0, 0};    // 0 empty, 1 expansion, 2 drain
        // enqueue the expansion (or the drain of parked keys) of round k into set k & 1
        auto enqueue_A = [&](u64 k) -> int {
            DistState::Set& S = D.set[k & 1];
            HIPCHK(c, hipStreamWaitEvent(c->st, S.ev_free, 0));
            HIPCHK(c, hipMemsetAsync(S.ocount, 0, 8 * (u64)(W + 1), c->st));
            DevBufs Bb = c->B;
            Bb.key_out = S.key_out;
            Bb.tick_out = S.tick_out;
            Bb.ocount = S.ocount;
            Bb.pool = S.pool;
            Bb.npool = S.ocount + W;
            Bb.pool_cap = D.pool_cap;
            round_states[k & 1] = 0;
            round_kind[k & 1] = 0;
            S.timed = 0;
            if (ovf_done < ovf_known) {
                const u64 n = std::min(kcap, ovf_known - ovf_done);
                HIPCHK(c, launch_drain(Bb, ovf_done, n, c->st));
                ovf_done += n;
                round_kind[k & 1] = 2;
            } else if (cursor < hi) {
                const u64 target = (u64)(D.fill * (double)kcap / std::max(rho, 0.02));
                // the rest of the level in equal rounds of at most this size (not full
                // rounds and a small remainder: a small round idles most of the grid)
                const u64 cap = std::max<u64>(1, std::min<u64>({1ull << kMaxLaunchLog2, target, split_cap}));
                const u64 rest = hi - cursor, nr = (rest + cap - 1) / cap;
                const u64 n = (rest + nr - 1) / nr;
                HIPCHK(c, hipEventRecord(S.k0, c->st));
                HIPCHK(c, launch(c->sh, 3, c->P, c->PT, Bb, cursor, cursor + n, nullptr, nullptr, 0, nullptr, c->st));
                // the pool flush's remote successors: keyed and routed to the outboxes
                if (W > 1 && !verify && !c->sh.sym)
                    HIPCHK(c, launch(c->sh, 14, c->P, c->PT, Bb, 0, 0, nullptr, nullptr, 0, nullptr, c->st));
                HIPCHK(c, hipEventRecord(S.k1, c->st));
                S.timed = 1;
                c->res.expand_launches += 1;
                cursor += n;
                round_states[k & 1] = n;
                round_kind[k & 1] = 1;
            }
            if (verify) {  // publish this round's local states, then check the hits deferred to them
                if (int rc = read_counters(c)) return rc;
                const u64 c1 = c->h_ctr->count;
                if (c1 > vpub)
                    HIPCHK(c, launch(c->sh, 5, c->P, c->PT, c->B, vpub, c1, nullptr, nullptr, 0, nullptr, c->st));
                vpub = c1;
                if (c->h_ctr->vcount) {
                    HIPCHK(c, launch(c->sh, 6, c->P, c->PT, c->B, c->h_ctr->vcount, 0, nullptr, nullptr, 0, nullptr, c->st));
                    HIPCHK(c, hipMemsetAsync(&c->B.ctr->vcount, 0, 8, c->st));
                }
            }
            HIPCHK(c, hipEventRecord(S.ev_exp, c->st));
            return 0;
        };
        std::vector<u64> soff((size_t)W), scnt((size_t)W), roff((size_t)W), rcnt((size_t)W);
        std::vector<u64> s2((size_t)W), o2((size_t)W), r2((size_t)W), q2((size_t)W);
        if (int rc = enqueue_A(0)) return rc;
        for (u64 k = 0;; ++k) {
            const int b = (int)(k & 1);
            DistState::Set& S = D.set[b];
            D.rnd = (int)k;
            const bool host_more = cursor < hi || ovf_done < ovf_known;
            // ---- count row of round k (after its expansion), on xs
            D.phase = "count all-to-all";
            if (W == 1) {
                // a world of one: the row is its own all-to-all; the pack kernel writes
                // it (both halves) straight into the pinned host row, on the ctx stream
                // right after the expansion: no stream hop, collective or copy
                HIPCHK(c, hipEventRecord(S.x0, c->st));
                DevBufs Bb = c->B;
                Bb.ocount = S.ocount;
                HIPCHK(c, launch_pack_counts(Bb, host_more ? 1ull : 0ull, ovf_done, S.h_cx, c->st,
                                             S.h_cx + RWD * (u64)W + 1));
                HIPCHK(c, hipEventRecord(D.ev_cnt, c->st));
            } else {
                HIPCHK(c, hipStreamWaitEvent(D.xs, S.ev_exp, 0));
                HIPCHK(c, hipEventRecord(S.x0, D.xs));
                {
                    DevBufs Bb = c->B;
                    Bb.ocount = S.ocount;
                    HIPCHK(c, launch_pack_counts(Bb, host_more ? 1ull : 0ull, ovf_done, S.cx, D.xs));
                }
                if (int rc = a2a_u64(c, S.cx, S.cx + RWD * (u64)W + 1, RWD)) return rc;
                HIPCHK(c, hipMemcpyAsync(S.h_cx, S.cx, row_len * 8, hipMemcpyDeviceToHost, D.xs));
                HIPCHK(c, hipEventRecord(D.ev_cnt, D.xs));
            }
            // the next round's expansion is queued before waiting, so the GPU
            // expands while the counts travel (not in RMC_DIST_OVERLAP=0 runs)
            bool next_queued = false;
            if (D.overlap && host_more) {
                if (int rc = enqueue_A(k + 1)) return rc;
                next_queued = true;
            }
            if (int rc = xwait(c, D.ev_cnt)) return rc;
            const u64* cx = S.h_cx;
            // a rank whose parking buffer overflowed says so in its flags (bit 1):
            // every rank sees every row and stops here alike
            for (int p = 0; p < W; ++p)
                if (rx(cx, p)[1] & 2u)
                    return fail(c, RMC_E_CAPACITY, "exchange parking buffer full on rank " + std::to_string(p) +
                                                       " (raise keys_per_dest) at " + where(c));
            const u64 novf = std::min(cx[RWD * (u64)W], c->B.ovf_cap);  // never drain past the buffer
            const u64 newly_parked = novf - std::min(novf, ovf_known);
            D.parked += newly_parked;
            ovf_known = std::max(ovf_known, novf);
            bool global_more = false, global_sends = false;
            u64 mx = 0, tot_in = 0;
            for (int p = 0; p < W; ++p) {
                global_more |= (rx(cx, p)[1] & 1u) != 0;
                global_sends |= (rx(cx, p)[1] & 4u) != 0;
                // phase-1 key records: the raw fingerprint (k, s32), KEYB bytes each
                scnt[(size_t)p] = cx[RWD * (u64)p] * KEYB;
                soff[(size_t)p] = (u64)p * kcap * KEYB;
                rcnt[(size_t)p] = rx(cx, p)[0] * KEYB;
                roff[(size_t)p] = tot_in * KEYB;
                tot_in += rx(cx, p)[0];
                mx = std::max(mx, cx[RWD * (u64)p]);
                D.keys_sent += cx[RWD * (u64)p];
            }
            if (S.timed) {
                c->res.expand_kernel_seconds += 1e-3 * elapsed_ms(S.k0, S.k1);
                S.timed = 0;
            }
            if (D.set[b ^ 1].xtimed) {  // the previous round is complete on xs (stream order)
                D.xfer_seconds += 1e-3 * elapsed_ms(D.set[b ^ 1].x0, D.set[b ^ 1].x1);
                D.set[b ^ 1].xtimed = 0;
            }
            if (round_kind[b] == 1 && round_states[b])  // keys per state of the fullest owner (parked ones included)
                rho = std::max(0.5 * rho, (double)(mx + newly_parked) / (double)round_states[b]);
            if (D.debug)
                fprintf(stderr, "[rmc rank %d] level %d round %llu kind %d states %llu: most keys to one owner %llu "
                                "(cap %llu), parked %llu/%llu, in %llu, rho %.3f, more %d\n",
                        me, depth, (unsigned long long)k, round_kind[b], (unsigned long long)round_states[b],
                        (unsigned long long)mx, (unsigned long long)kcap, (unsigned long long)ovf_done,
                        (unsigned long long)ovf_known, (unsigned long long)tot_in, rho, (int)global_more);
            if (tot_in > D.in_cap) return fail(c, RMC_E_CAPACITY, "phase-1 inbox full at " + where(c));
            if (global_more && !next_queued) {
                if (int rc = enqueue_A(k + 1)) return rc;
                next_queued = true;
            }
            // nothing crosses this rank this round (always so at one rank): no
            // phase 1 or 2 and no second read-back.  RCCL point-to-point groups
            // pair ranks, so the others go on without this one; the host
            // transport's all-to-all is a collective of every rank, so there
            // only a world of one skips.
            bool idle = !verify && (D.rccl || W == 1) && tot_in == 0;
            for (int p = 0; p < W; ++p) idle = idle && scnt[(size_t)p] == 0;
            if (idle) {
                hipStream_t is = W == 1 ? c->st : D.xs;  // where the count row ran
                HIPCHK(c, hipEventRecord(S.ev_free, is));
                HIPCHK(c, hipEventRecord(S.x1, is));
                S.xtimed = 1;
                D.chunks += 1;
                if (!global_more) {
                    // the level's last round and no rank sent keys in it: nothing
                    // changes a counter after its count row, so the rows carry
                    // every rank's final counters — no level-end all-gather
                    if (!global_sends && !verify) {
                        for (int p = 0; p < W; ++p) memcpy(&rows[(size_t)p], rx(cx, p) + 2, sizeof(Counters));
                        rows_final = true;
                    }
                    break;
                }
                continue;
            }
            // ---- phase 1: keys to their owners, replies back; phase 2 sizes
            D.phase = "phase 1 (keys to owners)";
            HIPCHK(c, hipMemsetAsync(D.sa, 0, 16 * (u64)W, D.xs));
            if (int rc = a2a(c, S.key_out, soff.data(), scnt.data(), D.key_in, roff.data(), rcnt.data())) return rc;
            SrcOff so{};
            for (int p = 0; p < W; ++p) so.o[p] = roff[(size_t)p] / KEYB;
            so.o[W] = tot_in;
            HIPCHK(c, launch_owner_insert(c->B, D.key_in, D.rep_out, tot_in, so, D.sa + W, D.xs));
            for (int p = 0; p < W; ++p) {  // block p of rep_out (keys from p) back to p; from d into rep_in + d * kcap
                s2[(size_t)p] = rcnt[(size_t)p] / KEYB;
                o2[(size_t)p] = roff[(size_t)p] / KEYB;
                r2[(size_t)p] = scnt[(size_t)p] / KEYB;
                q2[(size_t)p] = (u64)p * kcap;
            }
            D.phase = "phase 1 (replies)";
            if (int rc = a2a(c, D.rep_out, o2.data(), s2.data(), D.rep_in, q2.data(), r2.data())) return rc;
            if (mx) {
                DevBufs Bb = c->B;
                Bb.key_out = S.key_out;
                Bb.tick_out = S.tick_out;
                Bb.ocount = S.ocount;
                Bb.pool = S.pool;  // tickets POOL_TICK | index name this set's pool records
                HIPCHK(c, launch(c->sh, 8, c->P, c->PT, Bb, mx, 0, reinterpret_cast<const u32*>(D.rep_in), nullptr, 0,
                                 nullptr, D.xs));
            }
            HIPCHK(c, hipEventRecord(S.ev_free, D.xs));  // the set's keys and tickets are consumed
            HIPCHK(c, hipMemcpyAsync(D.h_sa, D.sa, 16 * (u64)W, hipMemcpyDeviceToHost, D.xs));
            HIPCHK(c, hipEventRecord(D.ev_acc, D.xs));
            if (int rc = xwait(c, D.ev_acc)) return rc;
            // ---- phase 2: the accepted states
            D.phase = "phase 2 (states to owners)";
            u64 tot_st = 0;
            for (int p = 0; p < W; ++p) {
                // verification ships every key's state (the seen ones to be compared)
                const u64 ns = D.h_sa[p], nr = verify ? rx(cx, p)[0] : D.h_sa[W + p];
                if (p != me && ns > kcap) return fail(c, RMC_E_HIP, "phase 2: more accepted states than keys sent");
                soff[(size_t)p] = (u64)p * kcap * RB;
                scnt[(size_t)p] = p == me ? 0 : ns * RB;
                rcnt[(size_t)p] = p == me ? 0 : nr * RB;
                roff[(size_t)p] = tot_st * RB;
                tot_st += rcnt[(size_t)p] / RB;
                if (p != me) D.states_sent += ns;
            }
            if (tot_st > (u64)W * kcap) return fail(c, RMC_E_CAPACITY, "phase-2 inbox full at " + where(c));
            if (int rc = a2a(c, c->B.st_out, soff.data(), scnt.data(), D.st_in, roff.data(), rcnt.data())) return rc;
            if (tot_st)
                HIPCHK(c, launch(c->sh, 9, c->P, c->PT, c->B, tot_st, 0, D.st_in, nullptr, 0, nullptr, D.xs));
            if (verify && tot_st) {  // publish the received new states, then compare the seen ones
                HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
                if (int rc = xwait(c, D.ev_h)) return rc;
                if (int rc = read_counters(c)) return rc;
                const u64 c2 = c->h_ctr->count;
                if (c2 > vpub)
                    HIPCHK(c, launch(c->sh, 5, c->P, c->PT, c->B, vpub, c2, nullptr, nullptr, 0, nullptr, D.xs));
                vpub = c2;
                HIPCHK(c, launch(c->sh, 11, c->P, c->PT, c->B, tot_st, 0, D.st_in, nullptr, 0, nullptr, D.xs));
                HIPCHK(c, hipEventRecord(D.ev_h, D.xs));
                if (int rc = xwait(c, D.ev_h)) return rc;
            }
            HIPCHK(c, hipEventRecord(S.x1, D.xs));
            S.xtimed = 1;
            D.chunks += 1;
            if (!global_more) break;
        }
        // expansion of the next level reads what xs stored: the ctx stream waits for it
        HIPCHK(c, hipEventRecord(D.ev_x, D.xs));
        HIPCHK(c, hipStreamWaitEvent(c->st, D.ev_x, 0));
        }
        if (int rc = level_end()) return rc;
        if (rep_timed) {  // a replicated level's launch (complete: the counters were gathered after it)
            c->res.expand_kernel_seconds += 1e-3 * elapsed_ms(D.set[0].k0, D.set[0].k1);
            rep_timed = false;
        }
        for (auto& S2 : D.set)  // exchange device time of the level's last round
            if (S2.xtimed) {
                D.xfer_seconds += 1e-3 * elapsed_ms(S2.x0, S2.x1);
                S2.xtimed = 0;
            }
        u64 tot = 0, gen = 0, pr = 0;
        for (int r = 0; r < W; ++r) {
            const Counters& k = rows[(size_t)r];
            tot += k.count;
            gen += k.generated;
            pr += k.probes;
            c->res.collisions += k.collisions;
            c->res.verified += k.vchecked;
        }
        const u64 nnew = tot - total_prev;
        total_prev = tot;
        generated += gen;
        probes += pr;
        // the next level's frontier on every rank: the states it stored in this one
        for (int r = 0; r < W; ++r) {
            fsz[(size_t)r] = rows[(size_t)r].count - count_before[(size_t)r];
            count_before[(size_t)r] = rows[(size_t)r].count;
        }
        c->level_start.push_back(c->h_ctr->count);
        if (nnew) ++depth;
        for (int r = 0; r < W && !c->have_target; ++r)  // the lowest rank's least violating index
            if (rows[(size_t)r].viol != ~0ull) {
                c->res.violated_inv = 1 << (int)(rows[(size_t)r].viol & 15);
                c->res.violation_depth = depth;
                c->have_target = 1;
                c->target_idx = ((u64)r << 48) | (rows[(size_t)r].viol >> 4);
            }
        if (!c->have_target && (c->cfg.flags & RMC_FLAG_CHECK_DEADLOCK))
            for (int r = 0; r < W && !c->have_target; ++r)
                if (rows[(size_t)r].deadlock != ~0ull) {
                    c->res.deadlock = 1;
                    c->have_target = 1;
                    c->target_idx = ((u64)r << 48) | rows[(size_t)r].deadlock;
                }
        if (any_cb) {  // progress: the same collective on every rank; all stop when rank 0's callback asks to
            rmc_level_stats ls{};
            ls.level = nnew ? depth - 1 : depth;
            ls.generated = generated;
            ls.distinct = tot;
            ls.new_states = nnew;
            ls.seconds = now_s() - t0;
            const int stop = (cb && cb(&ls, user)) ? 1 : 0;
            std::vector<int> votes((size_t)W);
            D.phase = "progress vote";
            if (int rc = allgather(c, &stop, sizeof stop, votes.data())) return rc;
            if (votes[0]) {
                c->res.left_on_queue = nnew;
                break;
            }
        }
        if (!nnew) break;
    }
    // ---- global summary
    c->res.generated = generated;
    c->res.distinct = total_prev;
    c->res.depth = depth;
    c->res.probes = probes;
    c->res.stored_here = c->level_start.back();
    c->res.keys_sent = D.keys_sent;
    c->res.states_sent = D.states_sent;
    c->res.chunks = D.chunks;
    c->res.exchange_seconds = D.xfer_seconds;
    c->res.exchange_wait_seconds = D.wait_seconds;
    c->res.parked = D.parked;
    const double Dd = (double)total_prev, G = (double)generated;
    c->res.collision_probability = fp_collision_estimate(Dd, G, c->table_slots, c->set_epoch != 0);
    c->res.seconds = now_s() - t0;
    D.phase = "done";
    return 0;
}

// Counterexample across ranks (TLC's distributed trace reconstruction): each
// step the rank holding the current state contributes {state, parent ref,
// lane} to an all-gather; the parent ref names the next rank.
int trace_sharded(rmc_ctx* c, rmc_state_view* states, int32_t* families, int32_t* instances, size_t cap,
                  size_t* len) {
    DistState& D = c->dist;
    const int W = D.world;
    const u64 RB = 8 * 2 + (u64)c->NW * 4;  // has | act, parent ref, state
    std::vector<uint8_t> mine(RB), all(RB * (u64)W);
    std::vector<std::vector<u32>> chain_states;
    std::vector<int> chain_act;
    u64 ref = c->target_idx;
    for (int guard = 0; guard < 100000; ++guard) {
        const int owner = (int)(ref >> 48);
        const u64 idx = ref & ((1ull << 48) - 1);
        std::fill(mine.begin(), mine.end(), 0);
        if (owner == D.rank) {
            u64 head[2] = {1, 0};
            uint8_t a = 0;
            HIPCHK(c, hipMemcpy(&head[1], c->B.parent + idx, 8, hipMemcpyDeviceToHost));
            HIPCHK(c, hipMemcpy(&a, c->B.act + idx, 1, hipMemcpyDeviceToHost));
            head[0] = 1 | ((u64)a << 8);
            memcpy(mine.data(), head, 16);
            HIPCHK(c, hipMemcpy(mine.data() + 16, c->B.store + idx * (u64)c->NW, (u64)c->NW * 4, hipMemcpyDeviceToHost));
        }
        if (int rc = allgather(c, mine.data(), RB, all.data())) return rc;
        const uint8_t* rec = all.data() + (u64)owner * RB;
        u64 head[2];
        memcpy(head, rec, 16);
        if (!(head[0] & 1)) return fail(c, RMC_E_HIP, "trace: rank " + std::to_string(owner) + " holds no state " +
                                                          std::to_string(idx));
        std::vector<u32> st((size_t)c->NW);
        memcpy(st.data(), rec + 16, (u64)c->NW * 4);
        chain_states.push_back(st);
        chain_act.push_back((int)((head[0] >> 8) & 0xFF));
        if (head[1] == ~0ull) break;
        ref = head[1];
    }
    std::reverse(chain_states.begin(), chain_states.end());
    std::reverse(chain_act.begin(), chain_act.end());
    *len = chain_states.size();
    for (size_t q = 0; q < chain_states.size() && q < cap; ++q) {
        if (states) decode_state(c, chain_states[q].data(), &states[q]);
        if (families) families[q] = family_of(c->P, chain_act[q]);
        if (instances) instances[q] = chain_act[q] == 255 ? -1 : chain_act[q];
    }
    return 0;
}

}  // namespace rmc_host

extern "C" {

int rmc_rccl_unique_id(uint8_t id[128]) {
    if (!id) return RMC_E_INVAL;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return RMC_E_HIP;
    static_assert(sizeof u == 128, "ncclUniqueId is 128 bytes");
    memcpy(id, &u, 128);
    return 0;
}

int rmc_shard(rmc_ctx* c, int32_t rank, int32_t world, const uint8_t* rccl_id, const rmc_transport* host,
              uint64_t keys_per_dest, uint64_t sent_cache_slots) {
    if (!c || world < 1 || world > kMaxWorld || rank < 0 || rank >= world) return RMC_E_INVAL;
    if (!rccl_id && !(host && host->alltoallv && host->allgather))
        return fail(c, RMC_E_INVAL, "rmc_shard needs an RCCL id or a host transport");
    if (c->spill.on) return fail(c, RMC_E_INVAL, "sharded mode does not support RMC_FLAG_SPILL");
    if (c->wide) return fail(c, RMC_E_INVAL, "sharded mode runs the packed layout only (bounds within its capacity)");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    free_dist(c);
    DistState& D = c->dist;
    D.rank = rank;
    D.world = world;
    D.rccl = rccl_id != nullptr;
    if (host) D.host = *host;
    const u64 W = (u64)world;
    // keys one round may send one owner: 2^26 keys over all owners by default
    // (2^25 at 2 ranks, 2^23 at 8), which bounds the outboxes and inboxes
    const u64 kcap = keys_per_dest ? keys_per_dest : std::min<u64>(1ull << 25, std::max<u64>(1ull << 20, (1ull << 26) / W));
    u64 slots = 1;
    while (slots < std::max<u64>(sent_cache_slots ? sent_cache_slots : (1ull << 27), 1024)) slots <<= 1;
    const u64 RB = (u64)(c->NW + 4) * 4;
    D.sent_slots = slots;
    D.in_cap = W * kcap;
    // (RMC_DIST_XPRIO=1: the exchange stream at the highest priority, A/B)
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    const char* xp = getenv("RMC_DIST_XPRIO");
    bool ok = hipStreamCreateWithPriority(&D.xs, hipStreamNonBlocking, (xp && atoi(xp)) ? prio_hi : prio_lo) ==
              hipSuccess;
    // full-state verification ships every remote successor: no sent-cache
    // (the default kernel keeps send markers in the fingerprint set instead)
    if (!c->sh.verify && c->sh.sym) ok = ok && hipMalloc(&c->B.sent, slots * 8) == hipSuccess;
    const u64 ovf_cap = std::max<u64>(W * kcap, 1ull << 20);  // parked keys per level: >= a round's worth
    ok = ok && hipMalloc(&c->B.ovf, ovf_cap * 24) == hipSuccess;  // {k, s32 | flags, ticket}
    // the pool flush's remote successors of one round: as many as the round's
    // outboxes hold (a fuller pool parks tickets); none leave a world of one
    D.pool_cap = world > 1 ? W * kcap : 64;
    for (auto& S : D.set) {
        ok = ok && hipMalloc(&S.key_out, W * kcap * KEYB) == hipSuccess && hipMalloc(&S.tick_out, W * kcap * 8) == hipSuccess &&
             hipMalloc(&S.ocount, 8 * (W + 1)) == hipSuccess && hipMalloc(&S.cx, 8 * (2 * kRowWords * W + 1)) == hipSuccess &&
             hipMalloc(&S.pool, D.pool_cap * RB) == hipSuccess &&
             hipHostMalloc(&S.h_cx, 8 * (2 * kRowWords * W + 1), hipHostMallocDefault) == hipSuccess;
        for (hipEvent_t* e : {&S.ev_exp, &S.ev_free})
            ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
        for (hipEvent_t* e : {&S.k0, &S.k1, &S.x0, &S.x1}) ok = ok && hipEventCreate(e) == hipSuccess;
    }
    for (hipEvent_t* e : {&D.ev_cnt, &D.ev_acc, &D.ev_c, &D.ev_x, &D.ev_h})
        ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
    // replicated levels: levels of at most rep_max states in total are gathered
    // whole on every rank (RMC_DIST_REP states; 0 turns them off)
    D.rep_max = 1ull << 20;
    if (const char* e = getenv("RMC_DIST_REP")) D.rep_max = std::min<u64>((u64)atoll(e), 1ull << 24);
    if (D.rep_max) {
        const u64 rbr = (u64)(c->NW + 6) * 4;
        ok = ok && hipMalloc(&D.rep_send, D.rep_max * rbr) == hipSuccess &&
             hipMalloc(&D.rep_buf, D.rep_max * rbr) == hipSuccess;
    }
    ok = ok && hipMalloc(&D.key_in, W * kcap * KEYB) == hipSuccess && hipMalloc(&D.rep_out, W * kcap) == hipSuccess &&
         hipMalloc(&D.rep_in, W * kcap) == hipSuccess && hipMalloc(&c->B.st_out, W * kcap * RB) == hipSuccess &&
         hipMalloc(&D.st_in, W * kcap * RB) == hipSuccess && hipMalloc(&D.sa, 16 * W) == hipSuccess &&
         hipHostMalloc(&D.h_sa, 16 * W, hipHostMallocDefault) == hipSuccess &&
         hipMalloc(&D.ag_dev, 4096 * (W + 1)) == hipSuccess;
    if (!ok) {
        free_dist(c);
        return fail(c, RMC_E_NOMEM, "sharded-mode buffers do not fit (lower keys_per_dest / sent_cache_slots)");
    }
    // send markers share the fingerprint set with this rank's states: twice the
    // slots keeps the load of linear probing near the single-GPU one (when
    // HBM allows; otherwise the set stays as rmc_create sized it)
    // (only with 8 GiB to spare after the larger set is allocated: the kernels'
    // scratch, RCCL and other ranks sharing the device allocate after this)
    size_t mfree = 0, mtot = 0;
    (void)hipMemGetInfo(&mfree, &mtot);
    if (world > 1 && !c->sh.verify && !c->sh.sym && !D.table_grown && mfree >= c->table_slots * 16 + (8ull << 30)) {
        u64* t2 = nullptr;
        if (hipMalloc(&t2, c->table_slots * 16) == hipSuccess) {
            (void)hipFree(c->B.table);
            c->B.table = t2;
            c->table_slots *= 2;
            c->B.tmask = c->table_slots - 1;
            c->set_epoch = 0;  // a new, uncleared set: the next run clears it
            D.table_grown = 1;
        }
    }
    D.ag_cap = 4096;
    D.debug = getenv("RMC_DIST_DEBUG") != nullptr;
    // rounds per large level: 4 at world > 1 (round 6; 2 before), so each round's
    // exchange overlaps the next round's expansion and only the last quarter of a
    // level's exchange is exposed; 1 at world 1, where no round exchanges anything
    // (283.4-283.7 vs 289.8-294.0 ms for 2 on the one-rank bench,
    // profiles/r04/ab/dist_split_r04u.txt)
    D.split = world > 1 ? 4 : 1;
    if (const char* s = getenv("RMC_DIST_SPLIT")) D.split = std::max(1, std::min(64, atoi(s)));
    if (const char* s = getenv("RMC_DIST_OVERLAP")) D.overlap = atoi(s) != 0;
    if (c->sh.verify) D.overlap = 0;  // rounds in order: each publishes its states before the next compares
    if (const char* s = getenv("RMC_DIST_FILL")) D.fill = std::max(0.01, std::min(64.0, atof(s)));
    c->B.smask = slots - 1;
    c->B.kcap = kcap;
    c->B.scap = kcap;
    c->B.scount = D.sa;
    c->B.ovf_cap = ovf_cap;
    c->B.rank = (u32)rank;
    c->B.world = (u32)world;
    c->B.ref_tag = (u64)rank << 48;
    const char* om = getenv("RMC_OWNER");  // partition: 0 fingerprint, 1 server-0 word, 2 servers 0+1
    c->B.owner_mode = om ? (u32)std::min(3, std::max(0, atoi(om))) : 2u;
    // SYMMETRY: the states of one orbit must meet at one owner, so the owner is
    // a function of the canonical fingerprint (server words differ across the orbit)
    if (c->sh.sym) c->B.owner_mode = 0;
    D.timeout_s = 300.0;
    if (const char* e = getenv("RMC_DIST_TIMEOUT_S")) D.timeout_s = std::max(0.1, atof(e));
    // test hook: rank RMC_DIST_STALL_RANK sleeps RMC_DIST_STALL_S (default twice
    // the deadline) before level RMC_DIST_STALL_LEVEL (default 2)
    D.stall_rank = -1;
    if (const char* e = getenv("RMC_DIST_STALL_RANK")) D.stall_rank = atoi(e);
    D.stall_level = 2;
    if (const char* e = getenv("RMC_DIST_STALL_LEVEL")) D.stall_level = atoi(e);
    D.stall_s = 2 * D.timeout_s;
    if (const char* e = getenv("RMC_DIST_STALL_S")) D.stall_s = atof(e);
    D.lvl = 0;
    D.rnd = 0;
    D.phase = "communicator init";
    if (D.rccl) {
        ncclUniqueId u;
        memcpy(&u, rccl_id, sizeof u);
        // non-blocking (RMC_DIST_NCCL_BLOCKING=1: the blocking mode, A/B): every
        // call is polled under the deadline, connection set-up included
        D.nonblocking = 1;
        if (const char* e = getenv("RMC_DIST_NCCL_BLOCKING")) D.nonblocking = atoi(e) ? 0 : 1;
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = D.nonblocking ? 0 : 1;
        // The whole set-up — the init call and, on the non-blocking communicator,
        // its completion — runs on a helper thread (on this ctx's device) that
        // lives until it is complete (RCCL's group state of a call is the calling
        // thread's), waited for here under the deadline: the call does not
        // promise to return at once for every bootstrap state (a peer that never
        // connects).  On expiry the helper, which owns the communicator, aborts it
        // itself once it leaves its poll loop (no other thread frees it while the
        // helper may still be polling it); this thread waits for that, bounded
        // (kAbortWait), and a call that never returns is left to the process exit.
        struct Init {
            std::atomic<int> done{0}, quit{0}, aborted{0};
            std::atomic<ncclComm_t> comm{nullptr};
            ncclResult_t r = ncclSuccess;
        };
        auto in = std::make_shared<Init>();
        const int dev = c->cfg.device;
        const bool nb = D.nonblocking != 0;
        std::thread([in, world, u, rank, cfg, dev, nb]() mutable {
            (void)hipSetDevice(dev);
            ncclComm_t cm = nullptr;
            ncclResult_t r = ncclCommInitRankConfig(&cm, world, u, rank, &cfg);
            in->comm.store(cm);
            while (nb && r == ncclInProgress && cm && !in->quit.load()) {
                ncclResult_t a = ncclSuccess;
                if (ncclCommGetAsyncError(cm, &a) != ncclSuccess) break;
                r = a;
                if (r == ncclInProgress) std::this_thread::sleep_for(std::chrono::microseconds(50));
            }
            if (in->quit.load() && cm) {  // the waiting thread gave up: the owner aborts
                (void)ncclCommAbort(cm);
                in->aborted.store(1);
            }
            in->r = r;
            in->done.store(1);
        }).detach();
        const double t_init = now_s();
        while (!in->done.load()) {
            if (now_s() - t_init > D.timeout_s) {
                in->quit.store(1);
                const double t_q = now_s();
                while (!in->done.load() && now_s() - t_q < kAbortWait)
                    std::this_thread::sleep_for(std::chrono::milliseconds(1));
                const bool returned = in->comm.load() != nullptr;
                bool aborted = in->aborted.load() != 0;
                if (in->done.load() && !aborted && returned) {
                    // the helper completed the init just before it saw quit: it has
                    // left the communicator, so it is aborted here
                    aborted = abort_bounded(in->comm.load());
                }
                D.comm = nullptr;  // never touched again by this thread
                const int rc = deadline_fail(c,
                                             returned ? "ncclCommInitRankConfig (waiting for every rank)"
                                                      : "ncclCommInitRankConfig (the call has not returned)",
                                             !returned || aborted ? 0 : 1);
                const std::string msg = c->err;
                free_dist(c);
                c->err = msg;
                return rc;
            }
            std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
        D.comm = in->comm.load();
        ncclResult_t r = in->r;
        if (r != ncclSuccess && r != ncclInProgress) {
            if (D.comm) (void)abort_bounded(D.comm);
            D.comm = nullptr;
            free_dist(c);
            return fail(c, RMC_E_HIP, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r));
        }
        if (int rc = nccl_done(c, r, "ncclCommInitRankConfig (waiting for every rank)")) {
            const std::string msg = c->err;
            free_dist(c);
            c->err = msg;
            return rc;
        }
    }
    D.on = 1;
    return 0;
}

}  // extern "C"
