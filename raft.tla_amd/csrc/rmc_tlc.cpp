// rmc_tlc.cpp — `rmc-tlc`, a drop-in for `java tlc2.TLC` on raft.tla models.
//
// Same command line shape as TLC (`[-workers N] [-config X.cfg] [-depth N]
// [-deadlock] X.tla`) and the same summary lines, so scripts that grep TLC's
// output ("states generated", "distinct states found", "depth of the complete
// state graph", "Error: Invariant ... is violated", "State N:") keep working.
// It is the host side above the C ABI (include/rmc.h); Java users bind the
// same symbols through Panama.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

#include "../../include/rmc.h"

namespace {

const char* kFamilies[10] = {"Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest",
                             "AdvanceCommitIndex", "AppendEntries", "Receive", "DuplicateMessage", "DropMessage"};
const char* kRoles[3] = {"Follower", "Candidate", "Leader"};
const char* kMtypes[4] = {"RequestVoteRequest", "RequestVoteResponse", "AppendEntriesRequest",
                          "AppendEntriesResponse"};

std::string srv(int i) { return "r" + std::to_string(i + 1); }
std::string val(int v) { return "v" + std::to_string(v + 1); }

std::string seq(const rmc_entry* e, int n) {
    if (n == 0) return "<<>>";
    std::string s = "<<";
    for (int x = 0; x < n; ++x) {
        if (x) s += ", ";
        s += "[term |-> " + std::to_string(e[x].term) + ", value |-> " + val(e[x].value) + "]";
    }
    return s + ">>";
}

template <class F>
std::string fn(int S, F f) {  // (r1 :> f(0) @@ r2 :> f(1) ...)
    std::string s = "(";
    for (int i = 0; i < S; ++i) {
        if (i) s += " @@ ";
        s += srv(i) + " :> " + f(i);
    }
    return s + ")";
}

std::string set_of(uint32_t m, int S) {
    std::string s = "{";
    bool first = true;
    for (int i = 0; i < S; ++i)
        if (m >> i & 1) { s += (first ? "" : ", ") + srv(i); first = false; }
    return s + "}";
}

std::string msg(const rmc_msg_view& m) {
    std::string s = "[mtype |-> " + std::string(kMtypes[m.mtype]) + ", mterm |-> " + std::to_string(m.mterm);
    switch (m.mtype) {
        case 0: s += ", mlastLogTerm |-> " + std::to_string(m.mlastLogTerm) + ", mlastLogIndex |-> " +
                     std::to_string(m.mlastLogIndex); break;
        case 1: s += std::string(", mvoteGranted |-> ") + (m.mvoteGranted ? "TRUE" : "FALSE") + ", mlog |-> " +
                     seq(m.mlog, m.mlog_len); break;
        case 2: s += ", mprevLogIndex |-> " + std::to_string(m.mprevLogIndex) + ", mprevLogTerm |-> " +
                     std::to_string(m.mprevLogTerm) + ", mentries |-> " + seq(m.mentries, m.mentries_len) +
                     ", mcommitIndex |-> " + std::to_string(m.mcommitIndex); break;
        default: s += std::string(", msuccess |-> ") + (m.msuccess ? "TRUE" : "FALSE") + ", mmatchIndex |-> " +
                      std::to_string(m.mmatchIndex);
    }
    return s + ", msource |-> " + srv(m.msource) + ", mdest |-> " + srv(m.mdest) + "]";
}

void print_state(const rmc_state_view& v) {
    const int S = v.n_servers;
    std::string bag = v.n_msgs ? "(" : "<<>>";
    for (int q = 0; q < v.n_msgs; ++q) {
        if (q) bag += " @@ ";
        bag += msg(v.msgs[q]) + " :> " + std::to_string(v.msgs[q].count);
    }
    if (v.n_msgs) bag += ")";
    printf("/\\ messages = %s\n", bag.c_str());
    printf("/\\ currentTerm = %s\n", fn(S, [&](int i) { return std::to_string(v.currentTerm[i]); }).c_str());
    printf("/\\ state = %s\n", fn(S, [&](int i) { return std::string(kRoles[v.state[i]]); }).c_str());
    printf("/\\ votedFor = %s\n",
           fn(S, [&](int i) { return v.votedFor[i] < 0 ? std::string("Nil") : srv(v.votedFor[i]); }).c_str());
    printf("/\\ log = %s\n", fn(S, [&](int i) { return seq(v.log[i], v.log_len[i]); }).c_str());
    printf("/\\ commitIndex = %s\n", fn(S, [&](int i) { return std::to_string(v.commitIndex[i]); }).c_str());
    printf("/\\ votesResponded = %s\n", fn(S, [&](int i) { return set_of(v.votesResponded[i], S); }).c_str());
    printf("/\\ votesGranted = %s\n", fn(S, [&](int i) { return set_of(v.votesGranted[i], S); }).c_str());
    printf("/\\ nextIndex = %s\n", fn(S, [&](int i) {
               return fn(S, [&](int j) { return std::to_string(v.nextIndex[i][j]); });
           }).c_str());
    printf("/\\ matchIndex = %s\n", fn(S, [&](int i) {
               return fn(S, [&](int j) { return std::to_string(v.matchIndex[i][j]); });
           }).c_str());
}

const char* inv_name(int bit) {
    switch (bit) {
        case RMC_INV_TYPEOK: return "TypeOK";
        case RMC_INV_ONE_LEADER: return "OneLeaderPerTerm";
        case RMC_INV_LOG_MATCHING: return "LogMatching";
        case RMC_INV_MESSAGES: return "MessagesInv";
        case RMC_INV_LEADER_VOTES: return "LeaderVotesQuorum";
        case RMC_INV_CAND_TERM: return "CandidateTermNotInLog";
        case RMC_INV_VOTES_GRANTED: return "VotesGrantedInv";
        case RMC_INV_QUORUM_LOG: return "QuorumLogInv";
        case RMC_INV_MORE_UP_TO_DATE: return "MoreUpToDateCorrect";
        case RMC_INV_LEADER_COMPLETE: return "LeaderCompleteness";
    }
    return "?";
}

// TLC's header of a behaviour step: the action of Next that produced the
// state and its location in raft.tla (the body of the action's definition;
// for Receive, the disjunct of raft.tla:393-403 that fired: UpdateTerm when
// the message's term is newer, else the one for its mtype).
std::string g_override_header;  // an override's action location (front-end notes), e.g. BugBecomeLeader

std::string step_header(int family, int instance, const rmc_state_view& parent) {
    if (family == 3 && !g_override_header.empty()) return g_override_header;
    std::string action = kFamilies[family], shown = action;
    if (family == 7) {
        const int S = parent.n_servers;
        const int q = instance - (6 * S + 2 * S * S);  // Receive lanes start after the server families
        if (q >= 0 && q < parent.n_msgs) {
            const rmc_msg_view& m = parent.msgs[q];
            if (m.mterm > parent.currentTerm[m.mdest]) action = shown = "UpdateTerm";
            else action = std::string("Receive:") + kMtypes[m.mtype];
        }
    }
    int32_t loc[4];
    if (rmc_action_location(action.c_str(), loc) != 0) return "<" + shown + ">";
    char buf[256];
    snprintf(buf, sizeof buf, "<%s line %d, col %d to line %d, col %d of module raft>", shown.c_str(), loc[0], loc[1],
             loc[2], loc[3]);
    return buf;
}

int progress(const rmc_level_stats* s, void*) {
    printf("Progress(%d) at %.2fs: %llu states generated, %llu distinct states found, %llu states left on queue.\n",
           s->level + 1, s->seconds, (unsigned long long)s->generated, (unsigned long long)s->distinct,
           (unsigned long long)s->new_states);
    fflush(stdout);
    return 0;
}

int usage() {
    fprintf(stderr,
            "usage: rmc-tlc [-config X.cfg] [-depth N] [-deadlock] [-device D] [-capacity N] [-workers N]\n"
            "               [-verify] [-fpseed S] [-checkpoint F] [-recover F] [-simulate [num=N]] [-seed S]\n"
            "               [-raft raft.tla] [-builtin-raft] [-gpus N] [-nospill] [-window N] [-fpmem B] X.tla\n"
            "  -gpus N        shard the search over N GPUs (one ctx and RCCL rank per GPU)\n"
            "  -raft F        the raft.tla to verify against the compiled-in spec (default: next to X.tla)\n"
            "  -builtin-raft  no raft.tla on disk: check the compiled-in lemmy/raft.tla (said in the output)\n"
            "  -depth N   stop after N BFS levels (level N is left on the queue)\n"
            "  -verify    full-state verification: compare every fingerprint hit with the stored state\n"
            "  -nospill   keep every state on the device (stop with a capacity error when it fills);\n"
            "             by default expanded levels spill to pinned host memory (single GPU)\n"
            "  -window N  states kept on the device when spilling (default: what the set leaves)\n"
            "  -fpseed S  fingerprint salt (TLC -fp: another member of the fingerprint family)\n"
            "  -fpmem B   bytes of HBM for the fingerprint set (TLC -fpmem; suffix K/M/G; it holds\n"
            "             B / 16 states, \"fingerprint set full\" past that); default: sized for the\n"
            "             largest store the device holds\n"
            "  -checkpoint F  write the search to F when it stops at -depth (TLC -checkpoint)\n"
            "  -recover F     continue the search saved in F (TLC -recover)\n"
            "  -simulate  random simulation (TLC -simulate; num=N behaviours, default 2^20;\n"
            "             -depth = states per behaviour, default 100; -seed = RNG seed)\n");
    return 2;
}

// TLC -simulate: random behaviours with the invariants checked on every state
// (Smokeraft.cfg:43-48 through rmc_sim_config_from_files).
int run_simulation(const std::string& cfg, const std::string& tla, const std::string& raft, uint32_t fopts, int device,
                   int depth, unsigned long long num, unsigned long long seed) {
    rmc_config c;
    rmc_sim_config sc;
    char info[2048];
    int rc = rmc_model_from_files(cfg.c_str(), tla.c_str(), raft.empty() ? nullptr : raft.c_str(),
                                  fopts | RMC_FRONT_SIMULATE, &c, &sc, info, sizeof info);
    if (rc) { printf("Error: %s\n", info); return 1; }
    if (info[0]) printf("%s\n", info);
    c.device = device;
    c.state_capacity = 1 << 12;  // no state store needed for walks
    if (depth > 0) sc.depth = depth;
    if (num > 0) sc.behaviours = num;
    sc.seed = seed;
    // a model that bounds no field (Smokeraft.cfg) walks on the wide layout with
    // TLC's draw (an action, then a successor); a bounded one within its bounds
    const bool wide = rmc_state_bytes(&c) > 64 * 4;
    if (wide) sc.mode = RMC_SIM_TLC;
    printf("Running Random Simulation with seed %llu: %llu behaviours of up to %d states, %s.\n",
           (unsigned long long)seed, (unsigned long long)sc.behaviours, sc.depth,
           sc.smoke_k ? "initial states from SmokeInit" : "initial state from Init");
    rmc_ctx* ctx = nullptr;
    rc = rmc_create(&c, &ctx);
    if (rc) { printf("Error: rmc_create failed (%d)\n", rc); return 1; }
    rmc_sim_result r;
    rc = rmc_simulate(ctx, &sc, &r);
    if (rc) { printf("Error: %s\n", rmc_last_error(ctx)); rmc_destroy(ctx); return 1; }
    if (sc.smoke_k) printf("SmokeInit: %llu initial states (k = %d).\n", (unsigned long long)r.init_states, sc.smoke_k);
    int exitcode = 0;
    if (r.violated_inv) {
        printf("Error: Invariant %s is violated.\n", inv_name(r.violated_inv));
        printf("Error: The behavior up to this point is:\n");
        std::vector<rmc_state_view> st((size_t)sc.depth);
        size_t len = 0;
        rmc_sim_replay(ctx, &sc, r.violation_behaviour, st.data(), st.size(), &len);
        for (size_t k = 0; k < len && k < st.size(); ++k) {
            printf("State %zu:\n", k + 1);
            print_state(st[k]);
            printf("\n");
        }
        exitcode = 12;
    } else {
        printf("No error has been found in %llu behaviours.\n", (unsigned long long)r.behaviours);
    }
    printf("%llu states generated (%llu steps), %llu behaviours truncated at the %s layout's capacity, "
           "%llu deadlocked (no successor within the capacity).\n",
           (unsigned long long)(r.steps + r.behaviours), (unsigned long long)r.steps,
           (unsigned long long)r.truncated, wide ? "wide" : "packed", (unsigned long long)r.deadlocked);
    printf("Finished in %.0fms (%.3g behaviours/s, %.3g steps/s on the device)\n", r.seconds * 1e3,
           r.behaviours / (r.kernel_seconds > 0 ? r.kernel_seconds : 1), r.steps / (r.kernel_seconds > 0 ? r.kernel_seconds : 1));
    rmc_destroy(ctx);
    return exitcode;
}

}  // namespace

int main(int argc, char** argv) {
    std::string cfg, tla;
    int depth = 0, device = 0, nodeadlock = 0, verify = 0;
    unsigned long long fpseed = 0, seed = 0, num = 0;
    int simulate = 0, gpus = 1;
    std::string ckpt, recover, raft;
    uint32_t fopts = 0;
    unsigned long long capacity = 0, window = 0, fpmem = 0;
    int nospill = 0;
    for (int a = 1; a < argc; ++a) {
        std::string s = argv[a];
        auto next = [&]() -> const char* { return a + 1 < argc ? argv[++a] : nullptr; };
        if (s == "-config") { const char* v = next(); if (!v) return usage(); cfg = v; }
        else if (s == "-depth") { const char* v = next(); if (!v) return usage(); depth = atoi(v); }
        else if (s == "-deadlock") nodeadlock = 1;  // TLC: -deadlock turns deadlock checking OFF
        else if (s == "-device") { const char* v = next(); if (!v) return usage(); device = atoi(v); }
        else if (s == "-capacity") { const char* v = next(); if (!v) return usage(); capacity = strtoull(v, nullptr, 10); }
        else if (s == "-workers") { if (!next()) return usage(); }  // accepted for compatibility
        else if (s == "-gpus") { const char* v = next(); if (!v) return usage(); gpus = atoi(v); }
        else if (s == "-verify") verify = 1;
        else if (s == "-nospill") nospill = 1;
        else if (s == "-fpmem") {
            const char* v = next();
            if (!v) return usage();
            char* e = nullptr;
            fpmem = strtoull(v, &e, 10);
            if (e && (*e == 'K' || *e == 'k')) fpmem <<= 10;
            else if (e && (*e == 'M' || *e == 'm')) fpmem <<= 20;
            else if (e && (*e == 'G' || *e == 'g')) fpmem <<= 30;
            else if (e && *e) return usage();
        }
        else if (s == "-window") { const char* v = next(); if (!v) return usage(); window = strtoull(v, nullptr, 10); }
        else if (s == "-raft") { const char* v = next(); if (!v) return usage(); raft = v; }
        else if (s == "-builtin-raft") fopts |= RMC_FRONT_BUILTIN_RAFT;
        else if (s == "-checkpoint") { const char* v = next(); if (!v) return usage(); ckpt = v; }
        else if (s == "-recover") { const char* v = next(); if (!v) return usage(); recover = v; }
        else if (s == "-simulate") {
            simulate = 1;
            if (a + 1 < argc && strncmp(argv[a + 1], "num=", 4) == 0) num = strtoull(argv[++a] + 4, nullptr, 10);
        }
        else if (s == "-seed") { const char* v = next(); if (!v) return usage(); seed = strtoull(v, nullptr, 0); }
        else if (s == "-fpseed" || s == "-fp") { const char* v = next(); if (!v) return usage(); fpseed = strtoull(v, nullptr, 0); }
        else if (s[0] == '-') { fprintf(stderr, "unsupported option %s\n", s.c_str()); return usage(); }
        else tla = s;
    }
    if (tla.empty()) return usage();
    if (cfg.empty()) cfg = (tla.size() > 4 && tla.substr(tla.size() - 4) == ".tla" ? tla.substr(0, tla.size() - 4) : tla) + ".cfg";
    printf("rmc-tlc: %s\n", rmc_version());
    if (const char* b = getenv("RMC_BUILTIN_RAFT")) if (b[0] == '1') fopts |= RMC_FRONT_BUILTIN_RAFT;
    if (simulate) return run_simulation(cfg, tla, raft, fopts, device, depth, num, seed);
    rmc_config c;
    char info[2048];
    // -depth N: a model that leaves fields unbounded (MCraft.cfg as shipped) runs level by level
    if (depth > 0) fopts |= RMC_FRONT_DEPTH_BOUNDED;
    int rc = rmc_model_from_files(cfg.c_str(), tla.c_str(), raft.empty() ? nullptr : raft.c_str(), fopts, &c, nullptr,
                                  info, sizeof info);
    if (rc) { printf("Error: %s\n", info); return 1; }
    if (info[0]) printf("%s\n", info);
    if (const char* a = strstr(info, "BecomeLeader <- "))
        if (const char* b = strstr(a, "; action <"))
            if (const char* e = strchr(b, '>')) g_override_header.assign(b + 9, e + 1);
    c.device = device;
    c.max_depth = depth;
    c.state_capacity = capacity;
    if (nodeadlock) c.flags &= ~RMC_FLAG_CHECK_DEADLOCK;
    if (verify) c.flags |= RMC_FLAG_VERIFY_STATES;
    // like TLC's states/ directory, expanded levels leave the device when it fills
    // (single GPU, packed layout; under -verify the spilled states keep a host copy
    // for the comparisons, and checkpoints of such runs stay resident; the wide
    // layout of -depth runs of unbounded models has no spill)
    if (!nospill && !(verify && (!ckpt.empty() || !recover.empty())) && gpus == 1 && rmc_state_bytes(&c) <= 64 * 4)
        c.flags |= RMC_FLAG_SPILL;
    c.device_window = window;
    c.set_bytes = fpmem;
    c.seed = fpseed;
    printf("Model: %d servers, %d values, CONSTRAINT MaxTerm=%d MaxLogLen=%d MaxMsgs=%d MaxDup=%d%s%s\n",
           c.n_servers, c.n_values, c.max_term, c.max_log_len, c.max_msgs, c.max_dup,
           (c.flags & RMC_FLAG_SYMMETRY) ? ", SYMMETRY Permutations(Server)" : "",
           (c.flags & RMC_FLAG_BUG_QUORUM) ? ", BecomeLeader quorum guard weakened" : "");
    if (c.invariants & (RMC_INV_VOTES_GRANTED | RMC_INV_QUORUM_LOG | RMC_INV_MORE_UP_TO_DATE | RMC_INV_LEADER_COMPLETE))
        printf("Note: Committed(i) is read as the first min(commitIndex[i], Len(log[i])) entries; raft.tla:896's "
               "SubSeq(log[i], 1, commitIndex[i]) is out of range when commitIndex[i] > Len(log[i]), which TLC "
               "would report as an evaluation error (specs/MCraftBounded.tla).\n");
    rmc_ctx* ctx = nullptr;
    rc = rmc_create(&c, &ctx);
    if (rc) { printf("Error: rmc_create failed (%d)\n", rc); return 1; }
    // -gpus N: one ctx per GPU (devices device..device+N-1), each a rank of the
    // sharded search on librmc's RCCL communicator, each driven by its own
    // thread through every collective (the BFS and the trace walk).  All
    // contexts are created before any communicator exists, and a rank that
    // fails later ends the process (stdout flushed, exit code 1) instead of
    // leaving the other ranks blocked in a collective.
    std::vector<rmc_state_view> tr_st;
    std::vector<int32_t> tr_fam, tr_inst;
    rmc_result r{};
    if (gpus > 1) {
        // -verify, -checkpoint and -recover work per rank: every rank compares
        // its own hits and writes / reads its own part, <F>.rank<r>
        std::vector<rmc_ctx*> ctxs((size_t)gpus, nullptr);
        ctxs[0] = ctx;
        for (int k = 1; k < gpus; ++k) {
            rmc_config cr = c;
            cr.device = device + k;
            if (rmc_create(&cr, &ctxs[(size_t)k])) {
                printf("Error: rank %d: rmc_create on device %d failed\n", k, cr.device);
                for (rmc_ctx* x : ctxs) rmc_destroy(x);
                return 1;
            }
        }
        uint8_t id[128];
        if (rmc_rccl_unique_id(id)) { printf("Error: rmc_rccl_unique_id failed\n"); return 1; }
        printf("Sharded over %d GPUs (librmc two-phase exchange over RCCL).\n", gpus);
        if (!recover.empty()) printf("Recovering from checkpoint %s.rank0..%d...\n", recover.c_str(), gpus - 1);
        else printf("Computing initial states...\n");
        fflush(stdout);
        std::atomic<int> done{0}, failed{-1};
        std::vector<std::string> errs((size_t)gpus);
        std::vector<std::thread> ranks;
        for (int k = 0; k < gpus; ++k) {
            ranks.emplace_back([&, k]() {
                rmc_ctx* h = ctxs[(size_t)k];
                auto bad = [&](const char* what) {
                    errs[(size_t)k] = std::string(what) + ": " + rmc_last_error(h);
                    int none = -1;
                    failed.compare_exchange_strong(none, k);
                };
                if (rmc_shard(h, k, gpus, id, nullptr, 0, 0)) { bad("rmc_shard"); return; }
                if (!recover.empty() && rmc_recover(h, recover.c_str())) { bad("rmc_recover"); return; }
                if (rmc_run_bfs(h, k == 0 ? progress : nullptr, nullptr)) { bad("rmc_run_bfs"); return; }
                rmc_result rr;
                rmc_get_result(h, &rr);
                if (!ckpt.empty() && rr.left_on_queue > 0 && !rr.violated_inv && !rr.deadlock &&
                    rmc_checkpoint(h, ckpt.c_str())) { bad("rmc_checkpoint"); return; }
                if (rr.violated_inv || rr.deadlock) {  // the trace walk is collective: every rank calls it
                    size_t n = 0;
                    if (rmc_trace(h, nullptr, nullptr, nullptr, 0, &n)) { bad("rmc_trace"); return; }
                    std::vector<rmc_state_view> st(n);
                    std::vector<int32_t> f(n), in(n);
                    if (rmc_trace(h, st.data(), f.data(), in.data(), n, &n)) { bad("rmc_trace"); return; }
                    if (k == 0) { tr_st.swap(st); tr_fam.swap(f); tr_inst.swap(in); }
                }
                done.fetch_add(1);
            });
        }
        while (done.load() < gpus && failed.load() < 0) std::this_thread::sleep_for(std::chrono::milliseconds(20));
        if (failed.load() >= 0) {
            printf("Error: rank %d: %s\n", failed.load(), errs[(size_t)failed.load()].c_str());
            fflush(stdout);
            fflush(stderr);
            _exit(1);  // the other ranks may be blocked in a collective of the failed one
        }
        for (auto& t : ranks) t.join();
        rmc_get_result(ctx, &r);
        for (int k = 1; k < gpus; ++k) rmc_destroy(ctxs[(size_t)k]);
    } else {
        if (!recover.empty()) {
            rc = rmc_recover(ctx, recover.c_str());
            if (rc) { printf("Error: %s\n", rmc_last_error(ctx)); rmc_destroy(ctx); return 1; }
            printf("Recovering from checkpoint %s...\n", recover.c_str());
        } else {
            printf("Computing initial states...\n");
        }
        rc = rmc_run_bfs(ctx, progress, nullptr);
        if (rc) { printf("Error: %s\n", rmc_last_error(ctx)); rmc_destroy(ctx); return 1; }
        rmc_get_result(ctx, &r);
        if (r.violated_inv || r.deadlock) {
            size_t len = 0;
            rmc_trace(ctx, nullptr, nullptr, nullptr, 0, &len);
            tr_st.resize(len);
            tr_fam.resize(len);
            tr_inst.resize(len);
            rmc_trace(ctx, tr_st.data(), tr_fam.data(), tr_inst.data(), len, &len);
        }
    }
    int exitcode = 0;
    if (r.violated_inv || r.deadlock) {
        if (r.violated_inv) printf("Error: Invariant %s is violated.\n", inv_name(r.violated_inv));
        else printf("Error: Deadlock reached.\n");
        printf("Error: The behavior up to this point is:\n");
        for (size_t k = 0; k < tr_st.size(); ++k) {
            if (tr_fam[k] < 0 || k == 0) printf("State %zu: <Initial predicate>\n", k + 1);
            else printf("State %zu: %s\n", k + 1, step_header(tr_fam[k], tr_inst[k], tr_st[k - 1]).c_str());
            print_state(tr_st[k]);
            printf("\n");
        }
        exitcode = 12;
    } else {
        printf("Model checking completed. No error has been found.\n");
        printf("  Estimates of the probability that TLC did not check all reachable states\n"
               "  because two distinct states had the same fingerprint:\n"
               "  calculated (optimistic):  val = %.1E\n", r.collision_probability);
    }
    if (verify) {
        printf("Full-state verification: %llu fingerprint hits compared state by state, %llu collisions.\n",
               (unsigned long long)r.verified, (unsigned long long)r.collisions);
        if (r.verified_spilled)
            printf("  (%llu of the hits were on states that had left the device window: compared with "
                   "their host copies)\n", (unsigned long long)r.verified_spilled);
    }
    printf("%llu states generated, %llu distinct states found, %llu states left on queue.\n",
           (unsigned long long)r.generated, (unsigned long long)r.distinct, (unsigned long long)r.left_on_queue);
    printf("The depth of the complete state graph search is %d.\n", r.depth);
    if (r.spills)
        printf("Spilled %llu expanded states out of the device window in %llu spills (%.2fs; trace links kept in %s).\n",
               (unsigned long long)r.spilled, (unsigned long long)r.spills, r.spill_seconds,
               r.spill_links_on_device ? "HBM" : "host memory");
    if (gpus > 1)
        printf("Exchange (rank 0): %llu rounds, %llu keys and %llu states sent, %llu keys parked, "
               "%.1fms of exchange on the device, %.1fms waited on the host.\n",
               (unsigned long long)r.chunks, (unsigned long long)r.keys_sent, (unsigned long long)r.states_sent,
               (unsigned long long)r.parked, r.exchange_seconds * 1e3, r.exchange_wait_seconds * 1e3);
    if (!ckpt.empty() && r.left_on_queue > 0 && !r.violated_inv && !r.deadlock) {
        if (gpus > 1) printf("Checkpoint written to %s.rank0..%d (%llu states on the queue).\n", ckpt.c_str(), gpus - 1,
                             (unsigned long long)r.left_on_queue);
        else if (rmc_checkpoint(ctx, ckpt.c_str())) printf("Error: %s\n", rmc_last_error(ctx));
        else printf("Checkpoint written to %s (%llu states on the queue).\n", ckpt.c_str(),
                    (unsigned long long)r.left_on_queue);
    }
    if (recover.empty())
        printf("Finished in %.0fms (%.0f distinct states/s)\n", r.seconds * 1e3, r.distinct / (r.seconds > 0 ? r.seconds : 1));
    else
        printf("Finished in %.0fms after recovery (counts include the checkpointed levels)\n", r.seconds * 1e3);
    rmc_destroy(ctx);
    return exitcode;
}
