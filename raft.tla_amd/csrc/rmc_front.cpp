// rmc_front.cpp — TLC model front-end for raft.tla (rmc_config_from_files).
//
// Reads the same files TLC reads (a root MC module + its .cfg, e.g.
// MCraft.tla / MCraft.cfg) and maps them to rmc_config.  This is not a TLA+
// parser: it recognises the constructs a raft.tla model uses:
//   cfg:  CONSTANT(S) `X = v` / `X <- Def`, SPECIFICATION, INIT/NEXT,
//         INVARIANT(S), CONSTRAINT(S), SYMMETRY, CHECK_DEADLOCK
//         (MCraft.cfg:1-39, Smokeraft.cfg:43-48);
//   tla:  `Name == body` definitions of the root module and of the modules it
//         EXTENDS that sit next to it (the standard modules and `raft` itself
//         are compiled in).
// Anything else is reported, by name, as unsupported (RMC_E_PARSE).
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <regex>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rmc.h"

namespace {

std::string slurp(const std::string& path, bool* ok) {
    std::ifstream f(path);
    *ok = (bool)f;
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// Strip \* line comments and (* *) block comments (nesting allowed).
std::string strip_comments(const std::string& s) {
    std::string o;
    int depth = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        if (i + 1 < s.size() && s[i] == '(' && s[i + 1] == '*') { ++depth; ++i; continue; }
        if (depth && i + 1 < s.size() && s[i] == '*' && s[i + 1] == ')') { --depth; ++i; continue; }
        if (depth) { if (s[i] == '\n') o += '\n'; continue; }
        if (i + 1 < s.size() && s[i] == '\\' && s[i + 1] == '*') {
            while (i < s.size() && s[i] != '\n') ++i;
            o += '\n';
            continue;
        }
        o += s[i];
    }
    return o;
}

std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && isspace((unsigned char)s[a])) ++a;
    while (b > a && isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

struct Module {
    std::map<std::string, std::string> defs;  // name -> body (params dropped)
    std::vector<std::string> extends;
};

const std::set<std::string> kStd = {"Naturals", "Integers", "Bags", "FiniteSets", "Sequences", "TLC",
                                    "Randomization", "TLCExt", "Reals"};

bool load_module(const std::string& dir, const std::string& name, std::map<std::string, Module>& mods,
                 std::string* err) {
    if (mods.count(name) || kStd.count(name) || name == "raft") return true;
    bool ok = false;
    std::string text = slurp(dir + "/" + name + ".tla", &ok);
    if (!ok) {
        *err = "cannot read module " + name + ".tla next to the cfg";
        return false;
    }
    text = strip_comments(text);
    // module body ends at the first line of 4+ '='
    std::regex endre("\n={4,}");
    std::smatch em;
    if (std::regex_search(text, em, endre)) text = text.substr(0, (size_t)em.position(0));
    Module M;
    std::smatch mm;
    std::regex extre("EXTENDS([^\\n]*)");
    if (std::regex_search(text, mm, extre)) {
        std::stringstream ss(mm[1].str());
        std::string tok;
        while (std::getline(ss, tok, ',')) {
            tok = trim(tok);
            if (!tok.empty()) M.extends.push_back(tok);
        }
    }
    // top-level definitions: identifier [ (params) ] == body, starting at column 0
    std::regex defre("(^|\\n)([A-Za-z_][A-Za-z0-9_]*)\\s*(\\([^)]*\\))?\\s*==");
    std::vector<std::pair<size_t, std::string>> starts;
    std::vector<size_t> body_at;
    for (auto it = std::sregex_iterator(text.begin(), text.end(), defre); it != std::sregex_iterator(); ++it) {
        starts.push_back({(size_t)it->position(0), (*it)[2].str()});
        body_at.push_back((size_t)(it->position(0) + it->length(0)));
    }
    for (size_t k = 0; k < starts.size(); ++k) {
        const size_t end = k + 1 < starts.size() ? starts[k + 1].first : text.size();
        std::string body = text.substr(body_at[k], end - body_at[k]);
        // a separator line (4+ dashes, MCraft.tla:6,11,16,21) ends a definition
        std::smatch sm;
        if (std::regex_search(body, sm, std::regex("\n[ \t]*-{4,}"))) body = body.substr(0, (size_t)sm.position(0));
        M.defs[starts[k].second] = trim(body);
    }
    mods[name] = M;
    for (const auto& e : M.extends)
        if (!load_module(dir, e, mods, err)) return false;
    return true;
}

struct Cfg {
    std::map<std::string, std::string> eq;     // X = v
    std::map<std::string, std::string> subst;  // X <- Def
    std::vector<std::string> invariants, constraints, symmetry, props, unknown;
    std::string spec, init, next, check_deadlock;
};

bool parse_cfg(const std::string& text, Cfg* c, std::string* err) {
    static const std::set<std::string> kw = {"CONSTANT", "CONSTANTS", "SPECIFICATION", "INIT", "NEXT",
                                             "INVARIANT", "INVARIANTS", "CONSTRAINT", "CONSTRAINTS",
                                             "SYMMETRY", "CHECK_DEADLOCK", "PROPERTY", "PROPERTIES",
                                             "VIEW", "ACTION_CONSTRAINT", "ACTION_CONSTRAINTS", "ALIAS",
                                             "POSTCONDITION"};
    std::vector<std::string> toks;
    {
        std::string t = strip_comments(text);
        std::string cur;
        for (size_t i = 0; i < t.size(); ++i) {
            const char ch = t[i];
            if (isspace((unsigned char)ch)) {
                if (!cur.empty()) toks.push_back(cur), cur.clear();
            } else if (ch == '=' && !(i + 1 < t.size() && t[i + 1] == '=')) {
                if (!cur.empty()) toks.push_back(cur), cur.clear();
                toks.push_back("=");
            } else if (ch == '<' && i + 1 < t.size() && t[i + 1] == '-') {
                if (!cur.empty()) toks.push_back(cur), cur.clear();
                toks.push_back("<-");
                ++i;
            } else {
                cur += ch;
            }
        }
        if (!cur.empty()) toks.push_back(cur);
    }
    std::string sec;
    for (size_t i = 0; i < toks.size(); ++i) {
        const std::string& t = toks[i];
        if (kw.count(t)) { sec = t; continue; }
        if (sec == "CONSTANT" || sec == "CONSTANTS") {
            if (i + 2 < toks.size() && (toks[i + 1] == "=" || toks[i + 1] == "<-")) {
                // a value may be a set literal spanning several tokens
                std::string v = toks[i + 2];
                size_t j = i + 2;
                if (v.size() && v[0] == '{') {
                    while (v.find('}') == std::string::npos && j + 1 < toks.size()) v += " " + toks[++j];
                }
                (toks[i + 1] == "=" ? c->eq : c->subst)[t] = v;
                i = j;
            } else {
                *err = "cfg: cannot read constant assignment near '" + t + "'";
                return false;
            }
        } else if (sec == "SPECIFICATION") c->spec = t;
        else if (sec == "INIT") c->init = t;
        else if (sec == "NEXT") c->next = t;
        else if (sec == "INVARIANT" || sec == "INVARIANTS") c->invariants.push_back(t);
        else if (sec == "CONSTRAINT" || sec == "CONSTRAINTS") c->constraints.push_back(t);
        else if (sec == "SYMMETRY") c->symmetry.push_back(t);
        else if (sec == "CHECK_DEADLOCK") c->check_deadlock = t;
        else if (sec == "PROPERTY" || sec == "PROPERTIES") c->props.push_back(t);
        else if (!sec.empty()) c->unknown.push_back(sec);
        else { *err = "cfg: token '" + t + "' outside any section"; return false; }
    }
    return true;
}

int count_set(const std::string& body) {  // "{r1, r2, r3}" -> 3
    std::string b = trim(body);
    if (b.size() < 2 || b.front() != '{' || b.back() != '}') return -1;
    b = trim(b.substr(1, b.size() - 2));
    if (b.empty()) return 0;
    int n = 1;
    for (char ch : b)
        if (ch == ',') ++n;
    return n;
}

}  // namespace

// sim != nullptr: a simulation model (Smokeraft.cfg:43-48): `Init <- SmokeInit`
// with `k` and `SmokeNat` from the modules (Smokeraft.tla:10-19), a StopAfter-
// style CONSTRAINT that is not a state bound (replaced by an explicit behaviour
// count), no state bounds required (only the packed capacity limits a walk).
static int parse_model(const char* cfg_path, const char* tla_path, rmc_config* out, rmc_sim_config* sim,
                       char* err, size_t err_cap) {
    std::string e;
    auto fail = [&](const std::string& m) {
        if (err && err_cap) snprintf(err, err_cap, "%s", m.c_str());
        return RMC_E_PARSE;
    };
    if (!cfg_path || !out) return fail("null argument");
    std::string cfgp = cfg_path;
    std::string dir = ".", stem = cfgp;
    const size_t sl = cfgp.find_last_of('/');
    if (sl != std::string::npos) { dir = cfgp.substr(0, sl); stem = cfgp.substr(sl + 1); }
    if (stem.size() > 4 && stem.substr(stem.size() - 4) == ".cfg") stem = stem.substr(0, stem.size() - 4);
    std::string root = stem;
    if (tla_path) {
        std::string tp = tla_path;
        const size_t s2 = tp.find_last_of('/');
        std::string tdir = s2 == std::string::npos ? "." : tp.substr(0, s2);
        root = s2 == std::string::npos ? tp : tp.substr(s2 + 1);
        if (root.size() > 4 && root.substr(root.size() - 4) == ".tla") root = root.substr(0, root.size() - 4);
        if (tdir != dir) dir = tdir;
    }
    bool ok = false;
    const std::string cfgtext = slurp(cfgp, &ok);
    if (!ok) return fail("cannot read " + cfgp);
    Cfg C;
    if (!parse_cfg(cfgtext, &C, &e)) return fail(e);
    std::map<std::string, Module> mods;
    if (!load_module(dir, root, mods, &e)) return fail(e);
    // does the root module reach raft?
    std::function<bool(const std::string&)> reaches = [&](const std::string& m) -> bool {
        if (m == "raft") return true;
        auto it = mods.find(m);
        if (it == mods.end()) return false;
        for (const auto& x : it->second.extends)
            if (reaches(x)) return true;
        return false;
    };
    if (!reaches(root)) return fail("module " + root + " does not EXTEND raft (directly or through a module next to it)");
    auto def = [&](const std::string& name, std::string* body) -> bool {
        for (auto& kv : mods) {
            auto it = kv.second.defs.find(name);
            if (it != kv.second.defs.end()) { *body = it->second; return true; }
        }
        return false;
    };
    auto value_of = [&](const std::string& name, std::string* v) -> bool {
        auto it = C.eq.find(name);
        if (it != C.eq.end()) { *v = it->second; return true; }
        auto is = C.subst.find(name);
        if (is != C.subst.end()) return def(is->second, v);
        return def(name, v);
    };
    auto int_of = [&](const std::string& tok, int* v) -> bool {
        std::string t = trim(tok), body;
        if (!t.empty() && (isdigit((unsigned char)t[0]) || t[0] == '-')) { *v = atoi(t.c_str()); return true; }
        if (value_of(t, &body)) {
            body = trim(body);
            if (!body.empty() && isdigit((unsigned char)body[0])) { *v = atoi(body.c_str()); return true; }
        }
        return false;
    };

    rmc_config g;
    memset(&g, 0, sizeof g);
    g.flags = RMC_FLAG_CHECK_DEADLOCK;
    std::string sv;
    if (!value_of("Server", &sv) || (g.n_servers = count_set(sv)) < 1)
        return fail("cannot resolve CONSTANT Server to a set literal of model values");
    if (!value_of("Value", &sv) || (g.n_values = count_set(sv)) < 1)
        return fail("cannot resolve CONSTANT Value to a set literal of model values");
    for (const char* mv : {"Follower", "Candidate", "Leader", "Nil", "RequestVoteRequest", "RequestVoteResponse",
                           "AppendEntriesRequest", "AppendEntriesResponse"}) {
        auto it = C.eq.find(mv);
        if (it != C.eq.end() && it->second != mv)
            return fail(std::string("CONSTANT ") + mv + " must be a model value");
    }
    // specification
    if (!C.spec.empty()) {
        std::string b;
        if (C.spec != "Spec" && !(def(C.spec, &b) && b.find("Init") != std::string::npos))
            return fail("SPECIFICATION " + C.spec + " is not raft's Spec");
    }
    if (!C.init.empty() && C.init != "Init") return fail("INIT " + C.init + " is not supported by BFS mode");
    if (!C.next.empty() && C.next != "Next") return fail("NEXT " + C.next + " is not supported");
    if (C.subst.count("Next")) return fail("Next override is not supported");
    if (sim) {
        memset(sim, 0, sizeof *sim);
        sim->behaviours = 1ull << 20;
        sim->depth = 100;  // TLC -simulate default depth
        sim->smoke_nat = 2;
        auto it = C.subst.find("Init");
        if (it != C.subst.end()) {
            std::string b;
            if (it->second != "SmokeInit" || !def("SmokeInit", &b))
                return fail("Init <- " + it->second + ": only Smokeraft's SmokeInit is compiled in");
            int kk = 0;
            if (!int_of("k", &kk) || kk < 1) return fail("SmokeInit needs `k == <number>` (Smokeraft.tla:17-19)");
            sim->smoke_k = kk;
            std::string nat;
            if (def("SmokeNat", &nat)) {
                std::smatch m;
                std::string nn;
                for (char ch : nat) if (!isspace((unsigned char)ch)) nn += ch;
                if (!std::regex_match(nn, m, std::regex("0\\.\\.([0-9]+)")))
                    return fail("SmokeNat must be 0..N (Smokeraft.tla:10-11)");
                sim->smoke_nat = atoi(m[1].str().c_str());
            }
        }
    } else if (C.subst.count("Init")) {
        return fail("Init overrides (e.g. Smokeraft's SmokeInit) are simulation-mode models (rmc-tlc -simulate)");
    }
    if (!C.props.empty()) return fail("PROPERTY " + C.props[0] + " (liveness) is out of scope");
    if (!C.unknown.empty()) return fail("cfg section " + C.unknown[0] + " is not supported");
    // BecomeLeader override (config 5 bug variant)
    auto bl = C.subst.find("BecomeLeader");
    if (bl != C.subst.end()) {
        std::string b;
        if (!def(bl->second, &b)) return fail("override BecomeLeader <- " + bl->second + ": definition not found");
        std::string nb;
        for (char ch : b) if (!isspace((unsigned char)ch)) nb += ch;
        if (nb.find("votesGranted[i]/={}") != std::string::npos && nb.find("\\inQuorum") == std::string::npos)
            g.flags |= RMC_FLAG_BUG_QUORUM;
        else
            return fail("override BecomeLeader <- " + bl->second + " is not the recognised quorum-weakening variant");
    }
    for (auto& kv : C.subst) {
        if (kv.first == "Server" || kv.first == "Value" || kv.first == "BecomeLeader") continue;
        if (sim && kv.first == "Init") continue;  // SmokeInit, resolved above
        std::string b;
        if (!def(kv.second, &b)) return fail("override " + kv.first + " <- " + kv.second + ": not found");
        int tmp;
        if (!int_of(b, &tmp)) return fail("override of " + kv.first + " is not supported");
    }
    // constraint -> bounds
    g.max_term = g.max_log_len = g.max_msgs = g.max_dup = -1;
    for (const auto& cn : C.constraints) {
        std::string b;
        if (!def(cn, &b)) return fail("CONSTRAINT " + cn + ": definition not found");
        std::string nb;
        for (char ch : b) if (!isspace((unsigned char)ch)) nb += ch;
        std::smatch m;
        struct Pat { const char* re; int32_t* dst; };
        const Pat pats[] = {
            {"currentTerm\\[[a-z]\\]<=([A-Za-z0-9_]+)", &g.max_term},
            {"Len\\(log\\[[a-z]\\]\\)<=([A-Za-z0-9_]+)", &g.max_log_len},
            {"Cardinality\\((?:DOMAINmessages|BagToSet\\(messages\\))\\)<=([A-Za-z0-9_]+)", &g.max_msgs},
            {"messages\\[[a-z]\\]<=([A-Za-z0-9_]+)", &g.max_dup},
        };
        int hits = 0;
        for (const auto& p : pats) {
            if (std::regex_search(nb, m, std::regex(p.re))) {
                int v;
                if (!int_of(m[1].str(), &v)) return fail("CONSTRAINT " + cn + ": bound " + m[1].str() + " is not a number");
                *p.dst = v;
                ++hits;
            }
        }
        if (!hits && sim) continue;  // e.g. StopAfter (Smokeraft.tla:84-92): a run budget, not a bound
        if (!hits) return fail("CONSTRAINT " + cn + " is not a recognised raft state bound");
    }
    if (sim) {  // unbounded fields: the packed capacity (rmc_simulate truncates beyond it)
        if (g.max_term < 0) g.max_term = 14;
        if (g.max_log_len < 0) g.max_log_len = 3;
        if (g.max_msgs < 0) g.max_msgs = 8;
        if (g.max_dup < 0) g.max_dup = 3;
    }
    if (g.max_term < 0 || g.max_log_len < 0 || g.max_msgs < 0 || g.max_dup < 0)
        return fail("the model is infinite without a CONSTRAINT bounding currentTerm, Len(log), "
                    "Cardinality(DOMAIN messages) and messages[m] (SURVEY.md §0.2)");
    for (const auto& in : C.invariants) {
        if (in == "TypeOK") g.invariants |= RMC_INV_TYPEOK;
        else if (in == "OneLeaderPerTerm") g.invariants |= RMC_INV_ONE_LEADER;
        else if (in == "LogMatching") g.invariants |= RMC_INV_LOG_MATCHING;
        else if (in == "MessagesInv") g.invariants |= RMC_INV_MESSAGES;
        else if (in == "LeaderVotesQuorum") g.invariants |= RMC_INV_LEADER_VOTES;
        else if (in == "CandidateTermNotInLog") g.invariants |= RMC_INV_CAND_TERM;
        else return fail("INVARIANT " + in + " is not compiled into the engine");
    }
    for (const auto& sy : C.symmetry) {
        std::string b;
        if (!def(sy, &b)) return fail("SYMMETRY " + sy + ": definition not found");
        std::string nb;
        for (char ch : b) if (!isspace((unsigned char)ch)) nb += ch;
        if (nb.rfind("Permutations(", 0) != 0) return fail("SYMMETRY " + sy + " is not Permutations(Server)");
        g.flags |= RMC_FLAG_SYMMETRY;
    }
    if (C.check_deadlock == "FALSE") g.flags &= ~RMC_FLAG_CHECK_DEADLOCK;
    *out = g;
    if (err && err_cap) err[0] = 0;
    return 0;
}

extern "C" int rmc_config_from_files(const char* cfg_path, const char* tla_path, rmc_config* out, char* err,
                                     size_t err_cap) {
    return parse_model(cfg_path, tla_path, out, nullptr, err, err_cap);
}

extern "C" int rmc_sim_config_from_files(const char* cfg_path, const char* tla_path, rmc_config* out,
                                         rmc_sim_config* sim, char* err, size_t err_cap) {
    if (!sim) {
        if (err && err_cap) snprintf(err, err_cap, "null argument");
        return RMC_E_PARSE;
    }
    return parse_model(cfg_path, tla_path, out, sim, err, err_cap);
}
