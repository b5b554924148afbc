// rmc_dist.cpp — sharded BFS over several GPUs behind the C ABI (rmc_shard).
//
// One ctx per GPU, each a rank of a fingerprint-space partition (SURVEY.md
// §8e; replaces TLC's distributed mode).  Per BFS level every rank expands the
// frontier it owns chunk by chunk; per chunk the exchange is two-phase:
//   phase 1  k_expand<DIST> puts the key of every successor owned elsewhere
//            (and not in the sent-cache) in that owner's key outbox, with a
//            local ticket (parent, lane); keys all-to-all; the owner inserts
//            them (k_owner_insert) and answers new/seen, 1 byte per key;
//            replies all-to-all (the reverse of the key exchange);
//   phase 2  k_materialize_remote re-derives the accepted successors from
//            their tickets into per-owner state outboxes; states all-to-all;
//            the owner stores them (k_store_remote).
// Collectives run on RCCL over xGMI (one communicator per ctx, on the ctx's
// stream) or on a caller-supplied host transport (gloo in the tests, where
// several ranks share one GPU).  Per chunk the host reads back two count
// vectors (the sizes RCCL's send/recv calls need) and all-gathers them.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "rmc_ctx.h"

using namespace rmc;
using namespace rmc_host;

namespace {

#define NCCLCHK(c, expr)                                                                         \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) return fail((c), RMC_E_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// All-to-all of per-peer byte blocks living on the device: block p of the send
// side is sbuf + soff[p] (scnt[p] bytes) for rank p; block p of the receive
// side lands at rbuf + roff[p] (rcnt[p] bytes) from rank p.
int a2a(rmc_ctx* c, const void* sbuf, const u64* soff, const u64* scnt, void* rbuf, const u64* roff, const u64* rcnt) {
    DistState& D = c->dist;
    const int W = D.world;
    if (D.rccl) {
        NCCLCHK(c, ncclGroupStart());
        for (int p = 0; p < W; ++p) {
            if (scnt[p]) NCCLCHK(c, ncclSend((const char*)sbuf + soff[p], scnt[p], ncclUint8, p, D.comm, c->st));
            if (rcnt[p]) NCCLCHK(c, ncclRecv((char*)rbuf + roff[p], rcnt[p], ncclUint8, p, D.comm, c->st));
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
                                     c->st));
        o += scnt[p];
    }
    HIPCHK(c, hipStreamSynchronize(c->st));
    if (D.host.alltoallv(D.host.user, D.stage_send.data(), scnt, D.stage_recv.data(), rcnt))
        return fail(c, RMC_E_HIP, "host transport alltoallv failed");
    o = 0;
    for (int p = 0; p < W; ++p) {
        if (rcnt[p])
            HIPCHK(c, hipMemcpyAsync((char*)rbuf + roff[p], D.stage_recv.data() + o, rcnt[p], hipMemcpyHostToDevice, c->st));
        o += rcnt[p];
    }
    HIPCHK(c, hipStreamSynchronize(c->st));
    return 0;
}

// All-gather of `bytes` host bytes per rank into all (world * bytes, rank order).
int allgather(rmc_ctx* c, const void* mine, u64 bytes, void* all) {
    DistState& D = c->dist;
    if (!D.rccl) {
        if (D.host.allgather(D.host.user, mine, bytes, all)) return fail(c, RMC_E_HIP, "host transport allgather failed");
        return 0;
    }
    const bool big = bytes > D.ag_cap;  // rows are small: the staging buffer is allocated once
    void* d_buf = D.ag_dev;
    if (big) HIPCHK(c, hipMallocAsync(&d_buf, bytes * (u64)(D.world + 1), c->st));
    char* d_in = (char*)d_buf + bytes * (u64)D.world;
    HIPCHK(c, hipMemcpyAsync(d_in, mine, bytes, hipMemcpyHostToDevice, c->st));
    NCCLCHK(c, ncclAllGather(d_in, d_buf, bytes, ncclUint8, D.comm, c->st));
    HIPCHK(c, hipMemcpyAsync(all, d_buf, bytes * (u64)D.world, hipMemcpyDeviceToHost, c->st));
    if (big) HIPCHK(c, hipFreeAsync(d_buf, c->st));
    HIPCHK(c, hipStreamSynchronize(c->st));
    return 0;
}

}  // namespace

namespace rmc_host {

void free_dist(rmc_ctx* c) {
    DistState& D = c->dist;
    (void)hipFree(c->B.sent);
    (void)hipFree(c->B.key_out);
    (void)hipFree(c->B.tick_out);
    (void)hipFree(c->B.ocount);
    (void)hipFree(c->B.st_out);
    (void)hipFree(c->B.scount);
    (void)hipFree(D.key_in);
    (void)hipFree(D.rep_out);
    (void)hipFree(D.rep_in);
    (void)hipFree(D.st_in);
    if (D.h_cnt) (void)hipHostFree(D.h_cnt);
    (void)hipFree(D.ag_dev);
    D.ag_dev = nullptr;
    D.ag_cap = 0;
    if (D.comm) (void)ncclCommDestroy(D.comm);
    c->B.sent = nullptr; c->B.key_out = nullptr; c->B.tick_out = nullptr; c->B.ocount = nullptr;
    c->B.st_out = nullptr; c->B.scount = nullptr;
    D.key_in = nullptr; D.rep_out = nullptr; D.rep_in = nullptr; D.st_in = nullptr; D.h_cnt = nullptr;
    D.comm = nullptr;
    D.on = 0;
}

int run_bfs_sharded(rmc_ctx* c, rmc_progress_fn cb, void* user) {
    DistState& D = c->dist;
    const int W = D.world, me = D.rank;
    const int RW = c->NW + 2;  // state record: packed state + global parent ref
    const double t0 = now_s();
    c->res = rmc_result{};
    c->level_start.clear();
    c->have_target = 0;
    D.keys_sent = D.states_sent = D.chunks = 0;
    D.xfer_seconds = 0;
    HIPCHK(c, hipMemsetAsync(c->B.table, 0, c->table_slots * 8, c->st));
    HIPCHK(c, hipMemsetAsync(c->B.sent, 0, D.sent_slots * 8, c->st));
    HIPCHK(c, set_fp_salt(c->cfg.seed, c->st));
    if (int rc = reset_counters(c, false)) return rc;
    // ---- Init (raft.tla:125-129): stored by its owner only
    {
        rmc_state_view iv;
        init_view(c->cfg, &iv);
        std::vector<u32> packed((size_t)c->NW);
        std::string why;
        if (encode_view(c, iv, packed.data(), &why)) return fail(c, RMC_E_INVAL, why);
        HIPCHK(c, hipMemcpyAsync(c->d_staged, packed.data(), packed.size() * 4, hipMemcpyHostToDevice, c->st));
        HIPCHK(c, launch(c->sh, 1, c->P, c->PT, c->B, 1, 0, c->d_staged, nullptr, 0, nullptr, c->st));
    }
    if (int rc = read_counters(c)) return rc;
    c->level_start.push_back(0);
    c->level_start.push_back(c->h_ctr->count);
    u64 generated = 1, probes = 0;
    int depth = 1;
    // level statistics, all-gathered: new, generated, probes, viol (index << 4 | bit, ~0 none),
    // deadlock index (~0 none), error flags
    struct LevelRow { u64 nnew, gen, probes, viol, dead, err, stored; };
    std::vector<LevelRow> rows((size_t)W);
    auto level_end = [&](u64 hi) -> int {
        const Counters& k = *c->h_ctr;
        LevelRow mine{k.count - hi, k.generated, k.probes, k.viol, k.deadlock,
                      (u64)(k.overflow | (k.table_full ? 16u : 0u)), k.count};
        const double tx = now_s();
        if (int rc = allgather(c, &mine, sizeof mine, rows.data())) return rc;
        D.xfer_seconds += now_s() - tx;
        for (int r = 0; r < W; ++r) {
            const u64 e = rows[(size_t)r].err;
            if (e & 16u) return fail(c, RMC_E_CAPACITY, "fingerprint set full on rank " + std::to_string(r));
            if (e & 2u) return fail(c, RMC_E_CAPACITY, "exchange outbox full on rank " + std::to_string(r) +
                                                       " (raise keys_per_dest)");
            if (e) return fail(c, RMC_E_CAPACITY, "state store full on rank " + std::to_string(r) +
                                                  " (raise rmc_config.state_capacity)");
        }
        return 0;
    };
    {  // Init's violation check (level 1)
        if (int rc = level_end(0)) return rc;
        for (int r = 0; r < W && !c->have_target; ++r)
            if (rows[(size_t)r].viol != ~0ull) {
                c->res.violated_inv = 1 << (int)(rows[(size_t)r].viol & 15);
                c->res.violation_depth = 1;
                c->have_target = 1;
                c->target_idx = ((u64)r << 48) | (rows[(size_t)r].viol >> 4);
            }
    }
    const u64 kcap = c->B.kcap, scap = c->B.scap;
    std::vector<u64> M((size_t)W * (W + 1)), soff((size_t)W), scnt((size_t)W), roff((size_t)W), rcnt((size_t)W);
    std::vector<u64> row((size_t)W + 1);
    const u64 nl = (u64)c->P.off[10];
    // Chunk sizing: rho = most keys one chunk sends one owner, per expanded
    // state.  It varies along a frontier (states received from other ranks are
    // appended after the local ones, and are of another kind) by up to ~1.6x
    // within a level (RMC_DIST_DEBUG logs of the bench model), so a chunk is sized
    // from the worst rho of the previous level and of this level so far, for an
    // outbox at most 40 % full.  An overflow is an error, never a silent drop.
    double rho_prev = (double)nl;
    while (!c->have_target) {
        const u64 lo = c->level_start[(size_t)depth - 1], hi = c->level_start[(size_t)depth];
        if (c->cfg.max_depth > 0 && depth >= c->cfg.max_depth) {
            u64 f = hi - lo;
            std::vector<u64> all((size_t)W);
            if (int rc = allgather(c, &f, 8, all.data())) return rc;
            c->res.left_on_queue = 0;
            for (u64 x : all) c->res.left_on_queue += x;
            break;
        }
        if (int rc = reset_counters(c, true)) return rc;
        u64 cursor = lo;
        double rho_lvl = 0;
        for (;;) {  // chunks: every rank takes part until no rank has frontier left
            const double rho = std::max({0.05, rho_prev, rho_lvl});
            const u64 chunk = std::max<u64>(1, (u64)((double)kcap / (2.5 * rho)));
            const u64 a = cursor, b = std::min(hi, a + chunk);
            HIPCHK(c, hipMemsetAsync(c->B.ocount, 0, 8 * (u64)W, c->st));
            if (a < b) {
                HIPCHK(c, hipEventRecord(c->ev0, c->st));
                HIPCHK(c, launch(c->sh, 3, c->P, c->PT, c->B, a, b, nullptr, nullptr, 0, nullptr, c->st));
                HIPCHK(c, hipEventRecord(c->ev1, c->st));
                c->res.expand_launches += 1;
            }
            HIPCHK(c, hipMemcpyAsync(D.h_cnt, c->B.ocount, 8 * (u64)W, hipMemcpyDeviceToHost, c->st));
            HIPCHK(c, hipStreamSynchronize(c->st));
            if (a < b) {
                float ms = 0.f;
                HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
                c->res.expand_kernel_seconds += 1e-3 * ms;
            }
            const double tx = now_s();
            u64 mx = 0;
            for (int d = 0; d < W; ++d) { row[(size_t)d] = D.h_cnt[d]; if (d != me) mx = std::max(mx, D.h_cnt[d]); }
            row[(size_t)W] = (b < hi ? 1u : 0u) | (mx > kcap ? 2u : 0u);
            if (D.debug)
                fprintf(stderr, "[rmc rank %d] level %d chunk [%llu, %llu) of [%llu, %llu): most keys to one owner %llu (cap %llu), rho %.3f\n",
                        me, depth, (unsigned long long)a, (unsigned long long)b, (unsigned long long)lo,
                        (unsigned long long)hi, (unsigned long long)mx, (unsigned long long)kcap, rho);
            if (int rc = allgather(c, row.data(), 8 * ((u64)W + 1), M.data())) return rc;
            bool more = false;
            u64 ph2 = 0;  // most keys one rank sent one owner: bounds the phase-2 rounds
            for (int r = 0; r < W; ++r) {
                const u64 f = M[(size_t)r * (W + 1) + W];
                if (f & 2u) return fail(c, RMC_E_CAPACITY, "phase-1 key outbox full on rank " + std::to_string(r) +
                                                           " (raise keys_per_dest)");
                more |= (f & 1u) != 0;
                for (int d = 0; d < W; ++d) if (d != r) ph2 = std::max(ph2, M[(size_t)r * (W + 1) + d]);
            }
            if (a < b) rho_lvl = std::max(rho_lvl, (double)std::max<u64>(mx, 1) / (double)(b - a));
            // ---- phase 1: keys to their owners, replies back
            u64 tot_in = 0;
            for (int p = 0; p < W; ++p) {
                soff[(size_t)p] = (u64)p * kcap * 8;
                scnt[(size_t)p] = p == me ? 0 : D.h_cnt[p] * 8;
                rcnt[(size_t)p] = p == me ? 0 : M[(size_t)p * (W + 1) + me] * 8;
                roff[(size_t)p] = tot_in * 8;
                tot_in += rcnt[(size_t)p] / 8;
                if (p != me) D.keys_sent += D.h_cnt[p];
            }
            if (tot_in > D.in_cap) return fail(c, RMC_E_CAPACITY, "phase-1 inbox full");
            if (ph2) {
                if (int rc = a2a(c, c->B.key_out, soff.data(), scnt.data(), D.key_in, roff.data(), rcnt.data())) return rc;
                HIPCHK(c, launch_owner_insert(c->B, D.key_in, D.rep_out, tot_in, c->st));
                // replies: block p of rep_out (keys from p) back to p; from d into rep_in + d * kcap
                std::vector<u64> s2((size_t)W), o2((size_t)W), r2((size_t)W), q2((size_t)W);
                for (int p = 0; p < W; ++p) {
                    s2[(size_t)p] = rcnt[(size_t)p] / 8;
                    o2[(size_t)p] = roff[(size_t)p] / 8;
                    r2[(size_t)p] = scnt[(size_t)p] / 8;
                    q2[(size_t)p] = (u64)p * kcap;
                }
                if (int rc = a2a(c, D.rep_out, o2.data(), s2.data(), D.rep_in, q2.data(), r2.data())) return rc;
                // ---- phase 2: accepted states, in rounds of at most scap per owner
                for (u64 w0 = 0; w0 < ph2; w0 += scap) {
                    HIPCHK(c, hipMemsetAsync(c->B.scount, 0, 8 * (u64)W, c->st));
                    HIPCHK(c, launch(c->sh, 8, c->P, c->PT, c->B, std::min(scap, ph2 - w0), w0,
                                     reinterpret_cast<const u32*>(D.rep_in), nullptr, 0, nullptr, c->st));
                    HIPCHK(c, hipMemcpyAsync(D.h_cnt + W, c->B.scount, 8 * (u64)W, hipMemcpyDeviceToHost, c->st));
                    HIPCHK(c, hipStreamSynchronize(c->st));
                    std::vector<u64> S2((size_t)W * W);
                    if (int rc = allgather(c, D.h_cnt + W, 8 * (u64)W, S2.data())) return rc;
                    u64 tot_st = 0;
                    const u64 RB = (u64)RW * 4;
                    for (int p = 0; p < W; ++p) {
                        soff[(size_t)p] = (u64)p * scap * RB;
                        scnt[(size_t)p] = p == me ? 0 : D.h_cnt[W + p] * RB;
                        rcnt[(size_t)p] = p == me ? 0 : S2[(size_t)p * W + me] * RB;
                        roff[(size_t)p] = tot_st * RB;
                        tot_st += rcnt[(size_t)p] / RB;
                        if (p != me) D.states_sent += D.h_cnt[W + p];
                    }
                    if (tot_st > (u64)W * scap) return fail(c, RMC_E_CAPACITY, "phase-2 inbox full");
                    if (int rc = a2a(c, c->B.st_out, soff.data(), scnt.data(), D.st_in, roff.data(), rcnt.data()))
                        return rc;
                    HIPCHK(c, launch(c->sh, 9, c->P, c->PT, c->B, tot_st, 0, D.st_in, nullptr, 0, nullptr, c->st));
                }
            }
            D.xfer_seconds += now_s() - tx;
            D.chunks += 1;
            cursor = b;
            if (!more) break;
        }
        if (rho_lvl > 0) rho_prev = rho_lvl;
        if (int rc = read_counters(c)) return rc;
        if (int rc = level_end(hi)) return rc;
        u64 nnew = 0, gen = 0, pr = 0;
        for (const auto& r : rows) { nnew += r.nnew; gen += r.gen; pr += r.probes; }
        generated += gen;
        probes += pr;
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
                if (rows[(size_t)r].dead != ~0ull) {
                    c->res.deadlock = 1;
                    c->have_target = 1;
                    c->target_idx = ((u64)r << 48) | rows[(size_t)r].dead;
                }
        {  // progress: the same collectives on every rank, with or without a callback;
           // all ranks stop together when rank 0's callback asks to
            rmc_level_stats ls{};
            ls.level = nnew ? depth - 1 : depth;
            ls.generated = generated;
            for (const auto& r : rows) ls.distinct += r.stored;
            ls.new_states = nnew;
            ls.seconds = now_s() - t0;
            const int stop = (cb && cb(&ls, user)) ? 1 : 0;
            std::vector<int> votes((size_t)W);
            if (int rc = allgather(c, &stop, sizeof stop, votes.data())) return rc;
            if (votes[0]) {
                c->res.left_on_queue = nnew;
                break;
            }
        }
        if (!nnew) break;
    }
    // ---- global summary
    u64 mine = c->level_start.back();
    std::vector<u64> all((size_t)W);
    if (int rc = allgather(c, &mine, 8, all.data())) return rc;
    u64 distinct = 0;
    for (u64 x : all) distinct += x;
    c->res.generated = generated;
    c->res.distinct = distinct;
    c->res.depth = depth;
    c->res.probes = probes;
    c->res.stored_here = mine;
    c->res.keys_sent = D.keys_sent;
    c->res.states_sent = D.states_sent;
    c->res.chunks = D.chunks;
    c->res.exchange_seconds = D.xfer_seconds;
    const double Dd = (double)distinct, G = (double)generated;
    c->res.collision_probability = Dd * (G - Dd) / 18446744073709551616.0;
    c->res.seconds = now_s() - t0;
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
    if (!c || world < 1 || world > 64 || rank < 0 || rank >= world) return RMC_E_INVAL;
    if (!rccl_id && !(host && host->alltoallv && host->allgather))
        return fail(c, RMC_E_INVAL, "rmc_shard needs an RCCL id or a host transport");
    if (c->sh.verify) return fail(c, RMC_E_INVAL, "sharded mode does not support full-state verification");
    if (c->spill.on) return fail(c, RMC_E_INVAL, "sharded mode does not support RMC_FLAG_SPILL");
    HIPCHK(c, hipSetDevice(c->cfg.device));
    free_dist(c);
    DistState& D = c->dist;
    D.rank = rank;
    D.world = world;
    D.rccl = rccl_id != nullptr;
    if (host) D.host = *host;
    const u64 W = (u64)world;
    const u64 kcap = keys_per_dest ? keys_per_dest : (1ull << 25);
    const u64 scap = std::max<u64>(kcap / 4, 1024);
    u64 slots = 1;
    while (slots < std::max<u64>(sent_cache_slots ? sent_cache_slots : (1ull << 27), 1024)) slots <<= 1;
    const u64 RB = (u64)(c->NW + 2) * 4;
    D.sent_slots = slots;
    D.in_cap = W * kcap;
    if (hipMalloc(&c->B.sent, slots * 8) != hipSuccess || hipMalloc(&c->B.key_out, W * kcap * 8) != hipSuccess ||
        hipMalloc(&c->B.tick_out, W * kcap * 8) != hipSuccess || hipMalloc(&c->B.ocount, 8 * W) != hipSuccess ||
        hipMalloc(&c->B.st_out, W * scap * RB) != hipSuccess || hipMalloc(&c->B.scount, 8 * W) != hipSuccess ||
        hipMalloc(&D.key_in, W * kcap * 8) != hipSuccess || hipMalloc(&D.rep_out, W * kcap) != hipSuccess ||
        hipMalloc(&D.rep_in, W * kcap) != hipSuccess || hipMalloc(&D.st_in, W * scap * RB) != hipSuccess ||
        hipHostMalloc(&D.h_cnt, 16 * W, hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&D.ag_dev, 4096 * (W + 1)) != hipSuccess) {
        free_dist(c);
        return fail(c, RMC_E_NOMEM, "sharded-mode buffers do not fit (lower keys_per_dest / sent_cache_slots)");
    }
    D.ag_cap = 4096;
    D.debug = getenv("RMC_DIST_DEBUG") != nullptr;
    c->B.smask = slots - 1;
    c->B.kcap = kcap;
    c->B.scap = scap;
    c->B.rank = (u32)rank;
    c->B.world = (u32)world;
    c->B.ref_tag = (u64)rank << 48;
    const char* om = getenv("RMC_OWNER");  // partition: 0 fingerprint, 1 server-0 word, 2 servers 0+1
    c->B.owner_mode = om ? (u32)std::min(2, std::max(0, atoi(om))) : 2u;
    // SYMMETRY: the states of one orbit must meet at one owner, so the owner is
    // a function of the canonical fingerprint (server words differ across the orbit)
    if (c->sh.sym) c->B.owner_mode = 0;
    if (D.rccl) {
        ncclUniqueId u;
        memcpy(&u, rccl_id, sizeof u);
        ncclResult_t r = ncclCommInitRank(&D.comm, world, u, rank);
        if (r != ncclSuccess) {
            free_dist(c);
            return fail(c, RMC_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
    }
    D.on = 1;
    return 0;
}

}  // extern "C"
