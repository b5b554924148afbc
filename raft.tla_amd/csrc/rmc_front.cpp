// rmc_front.cpp — TLC model front-end for raft.tla (rmc_model_from_files).
//
// Reads the files TLC reads (a root MC module, the modules it EXTENDS, its
// .cfg, and raft.tla itself) and maps them to rmc_config.  It is not a TLA+
// parser: the engine compiles one specification, so the front-end's job is to
// prove that the model on disk IS that specification, and to refuse it, by
// name, where it is not (DESIGN.md "Front-end"):
//   * raft.tla: every top-level unit of its module body (raft.tla:1-505) must
//     match the compiled-in digest (comments and whitespace normalised); the
//     one recognised edit is config 5's weakened BecomeLeader guard
//     (raft.tla:197), which sets RMC_FLAG_BUG_QUORUM;
//   * CONSTRAINT: split into top-level conjuncts; each must be a bound the
//     engine implements (currentTerm, Len(log), Cardinality(DOMAIN messages),
//     messages[m]), anything else is refused;
//   * INVARIANT / `BecomeLeader <-` / `Init <- SmokeInit`: the definition (with
//     the model definitions it uses) must be the compiled-in one;
//   * SYMMETRY: exactly Permutations(<the Server set>).
// The normalisation and digests follow tools/raft_digest.py, which generated
// model_digests.inc.
#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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

struct RaftUnit { const char* name; int line; uint64_t digest; };
struct KnownDef { const char* role; uint64_t digest; const char* source; };
struct ActionSpan { const char* action; int l1, c1, l2, c2; };
#include "model_digests.inc"

const char* kStateVars[] = {"messages", "currentTerm", "state", "votedFor", "log", "commitIndex",
                            "votesResponded", "votesGranted", "nextIndex", "matchIndex"};

uint64_t fnv(const std::string& s) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (unsigned char b : s) h = (h ^ b) * 0x100000001B3ull;
    return h;
}

std::string slurp(const std::string& path, bool* ok) {
    std::ifstream f(path);
    *ok = (bool)f;
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

bool file_exists(const std::string& p) {
    std::ifstream f(p);
    return (bool)f;
}

// Comments become spaces (newlines kept, so lines and columns stay), strings kept.
std::string strip_comments(const std::string& t) {
    std::string o;
    o.reserve(t.size());
    size_t i = 0, n = t.size();
    int depth = 0;
    bool in_str = false;
    while (i < n) {
        const char c = t[i];
        if (in_str) {
            o += c;
            if (c == '\\' && i + 1 < n) { o += t[i + 1]; i += 2; continue; }
            if (c == '"') in_str = false;
            ++i;
            continue;
        }
        if (depth == 0 && c == '"') { in_str = true; o += c; ++i; continue; }
        if (i + 1 < n && c == '(' && t[i + 1] == '*') { ++depth; o += "  "; i += 2; continue; }
        if (depth && i + 1 < n && c == '*' && t[i + 1] == ')') { --depth; o += "  "; i += 2; continue; }
        if (depth) { o += (c == '\n') ? '\n' : ' '; ++i; continue; }
        if (i + 1 < n && c == '\\' && t[i + 1] == '*') {
            while (i < n && t[i] != '\n') { o += ' '; ++i; }
            continue;
        }
        o += c;
        ++i;
    }
    return o;
}

std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && isspace((unsigned char)s[a])) ++a;
    while (b > a && isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

std::vector<std::string> split_lines(const std::string& s) {
    std::vector<std::string> out;
    size_t a = 0;
    for (;;) {
        const size_t b = s.find('\n', a);
        if (b == std::string::npos) { out.push_back(s.substr(a)); break; }
        out.push_back(s.substr(a, b - a));
        a = b + 1;
    }
    return out;
}

const std::regex kDefRe("^(LOCAL\\s+)?([A-Za-z_][A-Za-z0-9_]*)\\s*(\\([^)]*\\))?\\s*==");
const std::regex kKwRe("^(VARIABLES?|CONSTANTS?|ASSUME|AXIOM|EXTENDS|INSTANCE|THEOREM|LEMMA|RECURSIVE|USE|HIDE)\\b");
const std::regex kHdrRe("^\\s*-{4,}\\s*MODULE\\s+([A-Za-z_][A-Za-z0-9_]*)\\s*-{4,}\\s*$");
const std::regex kEndRe("^\\s*={4,}");
const std::regex kSepRe("^\\s*-{4,}\\s*$");

struct Unit {
    std::string name;  // definition name; "" for declarations / ASSUME / EXTENDS
    int line = 0;
    std::vector<std::pair<int, std::string>> lines;  // (1-based line, comment-stripped text)

    std::string norm() const {
        std::string out;
        bool first = true;
        for (const auto& [ln, s0] : lines) {
            std::string s = s0;
            for (char& ch : s) if (ch == '\t') ch = ' ';
            if (trim(s).empty()) continue;
            size_t ind = 0;
            while (ind < s.size() && s[ind] == ' ') ++ind;
            std::string content;
            {
                std::istringstream ss(s);
                std::string w;
                while (ss >> w) { if (!content.empty()) content += ' '; content += w; }
            }
            if (first && !name.empty()) {
                std::smatch m;
                if (std::regex_search(content, m, kDefRe))
                    content = trim(content.substr((size_t)m.position(2) + name.size()));
            }
            first = false;
            if (!out.empty()) out += '\n';
            out += std::to_string(ind) + "|" + content;
        }
        return out;
    }
    uint64_t digest() const { return fnv(norm()); }
    std::string text() const {
        std::string o;
        for (size_t k = 0; k < lines.size(); ++k) { if (k) o += '\n'; o += lines[k].second; }
        return o;
    }
    // the definition's body: the text after `==` on the first line, and the rest
    std::string body() const {
        std::string t = text();
        const size_t p = t.find("==");
        return p == std::string::npos ? t : t.substr(p + 2);
    }
    int body_line() const { return line; }
};

struct Module {
    std::string name, path;
    std::vector<std::string> extends;
    std::vector<Unit> units;
    std::map<std::string, size_t> defs;  // name -> unit index
};

bool parse_module(const std::string& path, Module* M, std::string* err) {
    bool ok = false;
    const std::string raw = slurp(path, &ok);
    if (!ok) { *err = "cannot read " + path; return false; }
    const std::vector<std::string> lines = split_lines(strip_comments(raw));
    size_t start = lines.size();
    for (size_t k = 0; k < lines.size(); ++k) {
        std::smatch m;
        if (std::regex_match(lines[k], m, kHdrRe)) { M->name = m[1].str(); start = k + 1; break; }
    }
    if (start == lines.size()) { *err = path + ": no `---- MODULE name ----` line"; return false; }
    M->path = path;
    long cur = -1;  // index of the open unit (units grows: no pointers into it)
    for (size_t k = start; k < lines.size(); ++k) {
        const std::string& s = lines[k];
        if (std::regex_search(s, kEndRe)) break;
        if (std::regex_match(s, kSepRe)) { cur = -1; continue; }
        if (!s.empty() && s[0] != ' ' && s[0] != '\t') {
            std::smatch dm;
            const bool kw = std::regex_search(s, kKwRe);
            const bool df = std::regex_search(s, dm, kDefRe);
            if (kw || df) {
                Unit u;
                u.line = (int)k + 1;
                u.name = (df && !kw) ? dm[2].str() : "";
                M->units.push_back(u);
                cur = (long)M->units.size() - 1;
            }
        }
        if (cur < 0) {
            if (!trim(s).empty()) {
                *err = path + ":" + std::to_string(k + 1) + ": text outside any definition or declaration";
                return false;
            }
            continue;
        }
        M->units[(size_t)cur].lines.push_back({(int)k + 1, s});
    }
    for (size_t q = 0; q < M->units.size(); ++q) {
        const Unit& u = M->units[q];
        if (!u.name.empty()) M->defs[u.name] = q;
        const std::string t = trim(u.text());
        if (u.name.empty() && t.rfind("EXTENDS", 0) == 0) {
            std::string rest = t.substr(7);
            for (char& ch : rest) if (ch == '\n') ch = ' ';
            std::stringstream ss(rest);
            std::string tok;
            while (std::getline(ss, tok, ',')) {
                tok = trim(tok);
                if (!tok.empty()) M->extends.push_back(tok);
            }
        }
    }
    return true;
}

std::set<std::string> idents(const std::string& text0) {
    std::string text;
    bool in_str = false;
    for (size_t i = 0; i < text0.size(); ++i) {  // drop string contents
        const char c = text0[i];
        if (in_str) {
            if (c == '\\' && i + 1 < text0.size()) { ++i; continue; }
            if (c == '"') { in_str = false; text += '"'; }
            continue;
        }
        if (c == '"') in_str = true;
        text += c;
    }
    std::set<std::string> out;
    auto word = [](char c) { return isalnum((unsigned char)c) || c == '_'; };
    for (size_t i = 0; i < text.size();) {
        const char c = text[i];
        if ((isalpha((unsigned char)c) || c == '_') && (i == 0 || !(word(text[i - 1]) || text[i - 1] == '\\'))) {
            size_t j = i;
            while (j < text.size() && word(text[j])) ++j;
            out.insert(text.substr(i, j - i));
            i = j;
        } else {
            ++i;
        }
    }
    return out;
}

const std::set<std::string> kStd = {"Naturals", "Integers", "Bags", "FiniteSets", "Sequences", "TLC",
                                    "Randomization", "TLCExt", "Reals"};

// ---- TLA+ tokens (for CONSTRAINT bodies) -------------------------------------------
struct Tok { std::string t; int line, col; };

std::vector<Tok> tokenize(const Unit& u, bool body_only) {
    std::vector<Tok> out;
    bool seen_eq = !body_only;
    static const char* multi[] = {"<=>", "|->", "/\\", "\\/", "=>", "<=", "=<", ">=", "/=", "==", "..", "->", "<<",
                                  ">>", ":>", "@@", "(+)", "(-)", "~>", "[]", "<>"};
    for (const auto& [ln, s] : u.lines) {
        size_t i = 0;
        while (i < s.size()) {
            const char c = s[i];
            if (isspace((unsigned char)c)) { ++i; continue; }
            Tok tk{"", ln, (int)i + 1};
            if (isalpha((unsigned char)c) || c == '_') {
                size_t j = i;
                while (j < s.size() && (isalnum((unsigned char)s[j]) || s[j] == '_')) ++j;
                tk.t = s.substr(i, j - i);
                i = j;
            } else if (isdigit((unsigned char)c)) {
                size_t j = i;
                while (j < s.size() && isdigit((unsigned char)s[j])) ++j;
                tk.t = s.substr(i, j - i);
                i = j;
            } else if (c == '"') {
                size_t j = i + 1;
                while (j < s.size() && s[j] != '"') j += (s[j] == '\\') ? 2 : 1;
                tk.t = s.substr(i, std::min(s.size(), j + 1) - i);
                i = j + 1;
            } else if (c == '\\' && i + 1 < s.size() && isalpha((unsigned char)s[i + 1])) {
                size_t j = i + 1;
                while (j < s.size() && isalpha((unsigned char)s[j])) ++j;
                tk.t = s.substr(i, j - i);
                i = j;
            } else {
                bool m = false;
                for (const char* op : multi) {
                    const size_t L = strlen(op);
                    if (s.compare(i, L, op) == 0) { tk.t = op; i += L; m = true; break; }
                }
                if (!m) { tk.t = std::string(1, c); ++i; }
            }
            if (!seen_eq) {
                if (tk.t == "==") seen_eq = true;
                continue;
            }
            out.push_back(tk);
        }
    }
    return out;
}

std::string join(const std::vector<Tok>& v, size_t a, size_t b) {
    std::string s;
    for (size_t k = a; k < b; ++k) { if (k > a) s += ' '; s += v[k].t; }
    return s;
}

bool is_open(const std::string& t) { return t == "(" || t == "[" || t == "{" || t == "<<"; }
bool is_close(const std::string& t) { return t == ")" || t == "]" || t == "}" || t == ">>"; }

// Split tokens [a, b) into top-level conjuncts: a bulleted /\ list (items at the
// first bullet's column), or an infix A /\ B /\ ... chain.  A disjunction or
// implication at the top, or a leading quantifier, keeps the range as one item.
std::vector<std::pair<size_t, size_t>> split_conj(const std::vector<Tok>& v, size_t a, size_t b) {
    std::vector<std::pair<size_t, size_t>> out;
    if (a >= b) return out;
    if (v[a].t == "/\\" || v[a].t == "\\land") {
        const int col = v[a].col;
        size_t st = a + 1;
        std::vector<std::pair<size_t, size_t>> items;
        for (size_t k = a + 1; k < b; ++k) {
            const bool first_on_line = v[k].line != v[k - 1].line;
            if ((v[k].t == "/\\" || v[k].t == "\\land") && v[k].col == col && first_on_line) {
                items.push_back({st, k});
                st = k + 1;
            }
        }
        items.push_back({st, b});
        for (const auto& [p, q] : items)  // an item may itself be a conjunction (infix or nested list)
            for (const auto& r : split_conj(v, p, q)) out.push_back(r);
        return out;
    }
    // a parenthesised whole: strip
    if (v[a].t == "(") {
        int d = 0;
        size_t k = a;
        for (; k < b; ++k) {
            if (is_open(v[k].t)) ++d;
            if (is_close(v[k].t) && --d == 0) break;
        }
        if (k == b - 1) return split_conj(v, a + 1, b - 1);
    }
    int d = 0;
    std::vector<size_t> cuts;
    for (size_t k = a; k < b; ++k) {
        const std::string& t = v[k].t;
        if (is_open(t)) { ++d; continue; }
        if (is_close(t)) { --d; continue; }
        if (d) continue;
        if (t == "\\/" || t == "\\lor" || t == "=>" || t == "<=>" || t == "\\equiv" || t == "~>")
            return {{a, b}};
        if (t == "\\A" || t == "\\E" || t == "\\AA" || t == "\\EE" || t == "LET" || t == "IF" || t == "CASE" ||
            t == "CHOOSE")
            break;  // extends to the end of the range
        if (t == "/\\" || t == "\\land") cuts.push_back(k);
    }
    size_t st = a;
    for (size_t c : cuts) { out.push_back({st, c}); st = c + 1; }
    out.push_back({st, b});
    return out;
}

struct Ctx {
    std::map<std::string, Module> mods;
    std::vector<std::string> mc;  // model modules (everything but raft and the standard modules), root first
    std::map<std::string, std::string> eq, subst;

    const Unit* def(const std::string& name, const Module** where = nullptr) const {
        for (const auto& mn : mc) {
            const Module& M = mods.at(mn);
            auto it = M.defs.find(name);
            if (it != M.defs.end()) {
                if (where) *where = &M;
                return &M.units[it->second];
            }
        }
        return nullptr;
    }
    uint64_t deep(const std::string& name, const std::set<std::string>& exclude, int depth = 0) const {
        const Unit* u = def(name);
        if (!u || depth > 64) return 0;
        std::string s;
        char buf[24];
        snprintf(buf, sizeof buf, "%016llx", (unsigned long long)u->digest());
        s = buf;
        for (const auto& r : idents(u->text())) {  // std::set: sorted, as the generator
            if (r == name || exclude.count(r) || !def(r)) continue;
            snprintf(buf, sizeof buf, "%016llx", (unsigned long long)deep(r, exclude, depth + 1));
            s += ";" + r + "=" + buf;
        }
        return fnv(s);
    }
    bool int_of(const std::string& tok, int* v) const {
        std::string t = trim(tok);
        if (!t.empty() && (isdigit((unsigned char)t[0]) || t[0] == '-')) {
            char* e = nullptr;
            const long x = strtol(t.c_str(), &e, 10);
            if (e && *e == 0) { *v = (int)x; return true; }
            return false;
        }
        auto it = eq.find(t);
        if (it != eq.end()) return int_of(it->second, v);
        auto is = subst.find(t);
        if (is != subst.end()) return int_of(is->second, v);
        const Unit* u = def(t);
        if (u) {
            const std::string b = trim(u->body());
            if (!b.empty() && isdigit((unsigned char)b[0])) return int_of(b, v);
        }
        return false;
    }
};

bool known_def(const char* role, uint64_t d, const char** src = nullptr) {
    for (const auto& k : kKnownDefs)
        if (strcmp(k.role, role) == 0 && k.digest == d) {
            if (src) *src = k.source;
            return true;
        }
    return false;
}

// The cfg file.
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
        const std::string t = strip_comments(text);
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
                std::string v = toks[i + 2];
                size_t j = i + 2;
                if (v.size() && v[0] == '{')
                    while (v.find('}') == std::string::npos && j + 1 < toks.size()) v += " " + toks[++j];
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

// "{r1, r2, r3}" -> element names (empty on a non-literal)
bool set_elems(const std::string& body, std::vector<std::string>* out) {
    std::string b = trim(body);
    if (b.size() < 2 || b.front() != '{' || b.back() != '}') return false;
    b = trim(b.substr(1, b.size() - 2));
    out->clear();
    if (b.empty()) return true;
    std::stringstream ss(b);
    std::string tok;
    while (std::getline(ss, tok, ',')) out->push_back(trim(tok));
    return true;
}

// raft.tla check: every unit of the module body against kRaftUnits.
int check_raft(const Module& R, uint32_t* flags, std::string* note, std::string* err) {
    std::map<std::string, uint64_t> want_defs;
    std::multiset<uint64_t> want_decls;
    std::map<std::string, int> want_line;
    for (const auto& u : kRaftUnits) {
        if (u.name[0]) { want_defs[u.name] = u.digest; want_line[u.name] = u.line; }
        else want_decls.insert(u.digest);
    }
    std::vector<std::string> bad;
    std::set<std::string> seen;
    bool bug = false;
    for (const Unit& u : R.units) {
        const uint64_t d = u.digest();
        if (u.name.empty()) {
            auto it = want_decls.find(d);
            if (it == want_decls.end()) bad.push_back("declaration at line " + std::to_string(u.line));
            else want_decls.erase(it);
            continue;
        }
        seen.insert(u.name);
        auto it = want_defs.find(u.name);
        if (it == want_defs.end()) {
            bad.push_back(u.name + " (line " + std::to_string(u.line) + ", not in lemmy/raft.tla)");
        } else if (it->second != d) {
            if (u.name == "BecomeLeader" && d == kBugBecomeLeaderDigest) bug = true;
            else bad.push_back(u.name + " (line " + std::to_string(u.line) + ", differs from raft.tla:" +
                               std::to_string(want_line[u.name]) + ")");
        }
    }
    for (const auto& kv : want_defs)
        if (!seen.count(kv.first)) bad.push_back(kv.first + " (missing; raft.tla:" + std::to_string(want_line[kv.first]) + ")");
    if (!want_decls.empty()) bad.push_back(std::to_string(want_decls.size()) + " declaration(s) of raft.tla missing or changed");
    if (!bad.empty()) {
        std::string m = R.path + " is not the raft.tla this engine compiles (lemmy/raft.tla:1-505): ";
        for (size_t k = 0; k < bad.size() && k < 6; ++k) m += (k ? "; " : "") + bad[k];
        if (bad.size() > 6) m += "; and " + std::to_string(bad.size() - 6) + " more";
        *err = m;
        return RMC_E_PARSE;
    }
    if (bug) *flags |= RMC_FLAG_BUG_QUORUM;
    *note = "raft.tla: " + R.path + " verified (" + std::to_string(R.units.size()) + " units match lemmy/raft.tla:1-505" +
            (bug ? "; BecomeLeader guard raft.tla:197 weakened -> bug variant" : "") + ")";
    return 0;
}

// TLC's location of an action defined by unit u: `<Name line L1, col C1 to
// line L2, col C2 of module M>` over the definition's body (rmc-tlc prints it
// as the trace header of the steps that action takes).
std::string body_location(const Unit& u, const std::string& name, const std::string& module) {
    int l1 = 0, c1 = 0, l2 = 0, c2 = 0;
    bool after = false;
    for (const auto& [ln, s] : u.lines) {
        size_t from = 0;
        if (!after) {
            const size_t p = s.find("==");
            if (p == std::string::npos) continue;
            from = p + 2;
            after = true;
        }
        const size_t q = s.find_first_not_of(" \t", from);
        if (q != std::string::npos && !l1) { l1 = ln; c1 = (int)q + 1; }
        const size_t e = s.find_last_not_of(" \t");
        if (l1 && e != std::string::npos && e + 1 > from) { l2 = ln; c2 = (int)e + 1; }
    }
    return "<" + name + " line " + std::to_string(l1) + ", col " + std::to_string(c1) + " to line " +
           std::to_string(l2) + ", col " + std::to_string(c2) + " of module " + module + ">";
}

struct Bounds { int term = -1, log = -1, msgs = -1, dup = -1; };

void set_min(int* dst, int v) { *dst = (*dst < 0 || v < *dst) ? v : *dst; }

}  // namespace

// options: RMC_FRONT_BUILTIN_RAFT (1) accept a model whose raft.tla is not on
// disk, using the compiled-in one; RMC_FRONT_SIMULATE (2) simulation model.
static int parse_model(const char* cfg_path, const char* tla_path, const char* raft_path, uint32_t options,
                       rmc_config* out, rmc_sim_config* sim, char* info, size_t info_cap) {
    std::string e;
    auto fail = [&](const std::string& m) {
        if (info && info_cap) snprintf(info, info_cap, "%s", m.c_str());
        return RMC_E_PARSE;
    };
    if (!cfg_path || !out) return fail("null argument");
    const std::string cfgp = cfg_path;
    std::string dir = ".", stem = cfgp;
    const size_t sl = cfgp.find_last_of('/');
    if (sl != std::string::npos) { dir = cfgp.substr(0, sl); stem = cfgp.substr(sl + 1); }
    if (stem.size() > 4 && stem.substr(stem.size() - 4) == ".cfg") stem = stem.substr(0, stem.size() - 4);
    std::string root = stem;
    if (tla_path) {
        const std::string tp = tla_path;
        const size_t s2 = tp.find_last_of('/');
        dir = s2 == std::string::npos ? "." : tp.substr(0, s2);
        root = s2 == std::string::npos ? tp : tp.substr(s2 + 1);
        if (root.size() > 4 && root.substr(root.size() - 4) == ".tla") root = root.substr(0, root.size() - 4);
    }
    bool ok = false;
    const std::string cfgtext = slurp(cfgp, &ok);
    if (!ok) return fail("cannot read " + cfgp);
    Cfg C;
    if (!parse_cfg(cfgtext, &C, &e)) return fail(e);

    // ---- modules: the root and every module it EXTENDS that sits next to it
    Ctx X;
    X.eq = C.eq;
    X.subst = C.subst;
    bool reaches_raft = false;
    std::function<bool(const std::string&)> load = [&](const std::string& name) -> bool {
        if (name == "raft") { reaches_raft = true; return true; }
        if (kStd.count(name) || X.mods.count(name)) return true;
        Module M;
        if (!parse_module(dir + "/" + name + ".tla", &M, &e)) {
            e = "module " + name + ": " + e;
            return false;
        }
        if (M.name != name) { e = dir + "/" + name + ".tla declares MODULE " + M.name; return false; }
        X.mods[name] = M;
        X.mc.push_back(name);
        for (const auto& x : X.mods[name].extends)
            if (!load(x)) return false;
        return true;
    };
    if (!load(root)) return fail(e);
    if (!reaches_raft) return fail("module " + root + " does not EXTEND raft (directly or through a module next to it)");

    uint32_t flags = RMC_FLAG_CHECK_DEADLOCK;
    std::vector<std::string> notes;
    // ---- raft.tla itself
    {
        std::string rp;
        if (raft_path && raft_path[0]) rp = raft_path;
        else if (const char* env = getenv("RMC_RAFT_TLA")) rp = env;
        else if (file_exists(dir + "/raft.tla")) rp = dir + "/raft.tla";
        if (!rp.empty()) {
            Module R;
            if (!parse_module(rp, &R, &e)) return fail(e);
            if (R.name != "raft") return fail(rp + " declares MODULE " + R.name + ", not raft");
            std::string note;
            if (int rc = check_raft(R, &flags, &note, &e)) return fail(e), rc;
            notes.push_back(note);
        } else if (options & RMC_FRONT_BUILTIN_RAFT) {
            notes.push_back("raft.tla: not found next to the model; using the compiled-in lemmy/raft.tla:1-505 "
                            "(RMC_FRONT_BUILTIN_RAFT)");
        } else {
            return fail("cannot find raft.tla next to " + root + ".tla (TLC needs it too): copy it there, set "
                        "RMC_RAFT_TLA, or accept the compiled-in lemmy/raft.tla explicitly (rmc-tlc -builtin-raft, "
                        "RMC_BUILTIN_RAFT=1)");
        }
    }
    for (const auto& mn : X.mc) {  // the model must not redefine raft's operators
        for (const auto& kv : X.mods[mn].defs) {
            for (const auto& u : kRaftUnits)
                if (u.name[0] && kv.first == u.name)
                    return fail("module " + mn + " redefines raft.tla's " + kv.first);
        }
    }

    auto value_of = [&](const std::string& name, std::string* v, std::string* via = nullptr) -> bool {
        auto it = C.eq.find(name);
        if (it != C.eq.end()) { *v = it->second; return true; }
        auto is = C.subst.find(name);
        if (is != C.subst.end()) {
            if (via) *via = is->second;
            const Unit* u = X.def(is->second);
            if (!u) return false;
            *v = u->body();
            return true;
        }
        const Unit* u = X.def(name);
        if (!u) return false;
        *v = u->body();
        return true;
    };

    rmc_config g;
    memset(&g, 0, sizeof g);
    std::string sv, server_via;
    std::vector<std::string> elems;
    if (!value_of("Server", &sv, &server_via) || !set_elems(sv, &elems) || elems.empty())
        return fail("cannot resolve CONSTANT Server to a set literal of model values");
    g.n_servers = (int)elems.size();
    if (std::set<std::string>(elems.begin(), elems.end()).size() != elems.size())
        return fail("CONSTANT Server lists a model value twice");
    if (!value_of("Value", &sv) || !set_elems(sv, &elems) || elems.empty())
        return fail("cannot resolve CONSTANT Value to a set literal of model values");
    g.n_values = (int)elems.size();
    if (std::set<std::string>(elems.begin(), elems.end()).size() != elems.size())
        return fail("CONSTANT Value lists a model value twice");
    for (const char* mv : {"Follower", "Candidate", "Leader", "Nil", "RequestVoteRequest", "RequestVoteResponse",
                           "AppendEntriesRequest", "AppendEntriesResponse"}) {
        auto it = C.eq.find(mv);
        if (it != C.eq.end() && it->second != mv) return fail(std::string("CONSTANT ") + mv + " must be a model value");
        if (C.subst.count(mv)) return fail(std::string("CONSTANT ") + mv + " must be a model value");
    }
    // ---- specification
    if (!C.spec.empty() && C.spec != "Spec") return fail("SPECIFICATION " + C.spec + " is not raft's Spec");
    if (!C.init.empty() && C.init != "Init") return fail("INIT " + C.init + " is not supported");
    if (!C.next.empty() && C.next != "Next") return fail("NEXT " + C.next + " is not supported");
    if (C.spec.empty() && C.init.empty()) return fail("the cfg names no SPECIFICATION (or INIT/NEXT)");
    const bool simulate = (options & RMC_FRONT_SIMULATE) != 0;
    if (simulate && !sim) return fail("null argument");
    if (simulate) {
        memset(sim, 0, sizeof *sim);
        sim->behaviours = 1ull << 20;
        sim->depth = 100;  // TLC -simulate default depth
        sim->smoke_nat = 2;
        auto it = C.subst.find("Init");
        if (it != C.subst.end()) {
            const std::set<std::string> ex = {"k", "SmokeNat"};
            const Unit* u = X.def(it->second);
            const char* src = nullptr;
            if (!u || !known_def("SmokeInit", X.deep(it->second, ex), &src))
                return fail("Init <- " + it->second + ": only Smokeraft's SmokeInit sampler (Smokeraft.tla:64-76) is "
                            "compiled in, and this definition is not it");
            int kk = 0;
            if (!X.int_of("k", &kk) || kk < 1) return fail("SmokeInit needs `k == <number>` (Smokeraft.tla:17-19)");
            sim->smoke_k = kk;
            if (const Unit* n = X.def("SmokeNat")) {
                std::string nn;
                for (char ch : n->body()) if (!isspace((unsigned char)ch)) nn += ch;
                std::smatch m;
                if (!std::regex_match(nn, m, std::regex("0\\.\\.([0-9]+)")))
                    return fail("SmokeNat must be 0..N (Smokeraft.tla:10-11)");
                sim->smoke_nat = atoi(m[1].str().c_str());
            } else {
                return fail("SmokeInit needs SmokeNat == 0..N (Smokeraft.tla:10-11)");
            }
            notes.push_back(std::string("Init <- ") + it->second + " (SmokeInit as in " + src + ", k = " +
                            std::to_string(kk) + ")");
        }
    } else if (C.subst.count("Init")) {
        return fail("Init overrides (e.g. Smokeraft's SmokeInit) are simulation models (rmc-tlc -simulate)");
    }
    if (!C.props.empty()) return fail("PROPERTY " + C.props[0] + " (liveness) is out of scope");
    if (!C.unknown.empty()) return fail("cfg section " + C.unknown[0] + " is not supported");
    // ---- overrides
    for (auto& kv : C.subst) {
        if (kv.first == "Server" || kv.first == "Value") continue;
        if (simulate && kv.first == "Init") continue;  // SmokeInit, resolved above
        if (kv.first == "BecomeLeader") {
            if (!X.def(kv.second)) return fail("override BecomeLeader <- " + kv.second + ": definition not found");
            if (!known_def("BecomeLeader", X.deep(kv.second, {})))
                return fail("override BecomeLeader <- " + kv.second +
                            " is not the compiled-in bug variant (specs/MCraftBounded.tla BugBecomeLeader: the "
                            "raft.tla:197 quorum guard weakened to votesGranted[i] /= {})");
            flags |= RMC_FLAG_BUG_QUORUM;
            const Module* where = nullptr;
            const Unit* u = X.def(kv.second, &where);
            notes.push_back("BecomeLeader <- " + kv.second + " (quorum guard weakened); action " +
                            body_location(*u, kv.second, where->name));
            continue;
        }
        int tmp;
        if (!X.int_of(kv.second, &tmp))
            return fail("override " + kv.first + " <- " + kv.second + " is not supported (the engine compiles raft.tla's " +
                        kv.first + ")");
    }
    // ---- CONSTRAINT -> bounds
    Bounds bd;
    const std::string server_set = server_via;  // `\A i \in <Server or its set definition>`
    std::function<int(const std::string&, const Unit&, const std::vector<Tok>&, size_t, size_t, int)> item;
    auto atom_bound = [&](const std::vector<Tok>& v, size_t a, size_t b, const std::string& var, int* dst_kind,
                          int* val) -> bool {
        // currentTerm [ v ] OP N  |  Len ( log [ v ] ) OP N
        auto opval = [&](size_t k) -> bool {
            if (k + 2 != b) return false;
            const std::string& op = v[k].t;
            int n;
            if (!X.int_of(v[k + 1].t, &n)) return false;
            if (op == "<=" || op == "=<" || op == "\\leq") { *val = n; return true; }
            if (op == "<") { *val = n - 1; return true; }
            return false;
        };
        if (b - a >= 6 && v[a].t == "currentTerm" && v[a + 1].t == "[" && v[a + 2].t == var && v[a + 3].t == "]")
            return opval(a + 4) && (*dst_kind = 0, true);
        if (b - a >= 9 && v[a].t == "Len" && v[a + 1].t == "(" && v[a + 2].t == "log" && v[a + 3].t == "[" &&
            v[a + 4].t == var && v[a + 5].t == "]" && v[a + 6].t == ")")
            return opval(a + 7) && (*dst_kind = 1, true);
        return false;
    };
    item = [&](const std::string& cname, const Unit& u, const std::vector<Tok>& v, size_t a, size_t b,
               int depth) -> int {
        const std::string txt = join(v, a, b);
        auto refuse = [&](const std::string& why) {
            e = "CONSTRAINT " + cname + ": conjunct `" + txt + "` (line " +
                std::to_string(a < v.size() ? v[a].line : u.line) + ") " + why;
            return RMC_E_PARSE;
        };
        if (a >= b) return refuse("is empty");
        if (depth > 16) return refuse("nests too deeply");
        if (v[a].t == "(") {  // a parenthesised conjunct: its own conjuncts
            int dd = 0;
            size_t k = a;
            for (; k < b; ++k) {
                if (is_open(v[k].t)) ++dd;
                if (is_close(v[k].t) && --dd == 0) break;
            }
            if (k == b - 1) {
                for (const auto& [p, q] : split_conj(v, a + 1, b - 1))
                    if (int rc = item(cname, u, v, p, q, depth + 1)) return rc;
                return 0;
            }
        }
        // a definition reference: splice its conjuncts
        if (b - a == 1 && (isalpha((unsigned char)v[a].t[0]) || v[a].t[0] == '_')) {
            const Unit* d = X.def(v[a].t);
            if (!d) return refuse("names no definition of the model");
            const std::set<std::string> ids = idents(d->body());
            bool touches_state = false;
            for (const char* sv2 : kStateVars) touches_state |= ids.count(sv2) > 0;
            if (!touches_state && (ids.count("TLCGet") || ids.count("TLCSet"))) {
                if (!simulate)
                    return refuse("is a run budget (TLCGet/TLCSet), not a state bound: BFS mode does not support it");
                notes.push_back("CONSTRAINT " + v[a].t + ": run budget, replaced by the behaviour count");
                return 0;
            }
            const std::vector<Tok> bt = tokenize(*d, true);
            for (const auto& [p, q] : split_conj(bt, 0, bt.size()))
                if (int rc = item(v[a].t, *d, bt, p, q, depth + 1)) return rc;
            return 0;
        }
        // \A v \in Server : <conjunction of currentTerm / Len(log) bounds>
        if (b - a >= 6 && v[a].t == "\\A" && v[a + 2].t == "\\in" && v[a + 4].t == ":" &&
            (v[a + 3].t == "Server" || (!server_set.empty() && v[a + 3].t == server_set))) {
            const std::string var = v[a + 1].t;
            for (const auto& [p, q] : split_conj(v, a + 5, b)) {
                int kind = -1, val = 0;
                if (!atom_bound(v, p, q, var, &kind, &val))
                    return refuse("has a part `" + join(v, p, q) +
                                  "` that is not currentTerm[" + var + "] <= N or Len(log[" + var + "]) <= N");
                set_min(kind == 0 ? &bd.term : &bd.log, val);
            }
            return 0;
        }
        // \A m \in DOMAIN messages : messages[m] <= N
        if (b - a == 12 && v[a].t == "\\A" && v[a + 2].t == "\\in" && v[a + 3].t == "DOMAIN" &&
            v[a + 4].t == "messages" && v[a + 5].t == ":" && v[a + 6].t == "messages" && v[a + 7].t == "[" &&
            v[a + 8].t == v[a + 1].t && v[a + 9].t == "]") {
            int n;
            const std::string& op = v[a + 10].t;
            if (!X.int_of(v[a + 11].t, &n)) return refuse("bound " + v[a + 11].t + " is not a number");
            if (op == "<=" || op == "=<" || op == "\\leq") set_min(&bd.dup, n);
            else if (op == "<") set_min(&bd.dup, n - 1);
            else return refuse("is not messages[m] <= N");
            return 0;
        }
        // Cardinality(DOMAIN messages) <= N   (or BagToSet(messages))
        if (b - a >= 7 && v[a].t == "Cardinality" && v[a + 1].t == "(") {
            size_t k = a + 2;
            if (v[k].t == "DOMAIN" && v[k + 1].t == "messages" && v[k + 2].t == ")") k += 3;
            else if (b - a >= 9 && v[k].t == "BagToSet" && v[k + 1].t == "(" && v[k + 2].t == "messages" &&
                     v[k + 3].t == ")" && v[k + 4].t == ")")
                k += 5;
            else return refuse("is not Cardinality(DOMAIN messages) <= N");
            if (k + 2 != b) return refuse("is not Cardinality(DOMAIN messages) <= N");
            int n;
            if (!X.int_of(v[k + 1].t, &n)) return refuse("bound " + v[k + 1].t + " is not a number");
            if (v[k].t == "<=" || v[k].t == "=<" || v[k].t == "\\leq") set_min(&bd.msgs, n);
            else if (v[k].t == "<") set_min(&bd.msgs, n - 1);
            else return refuse("is not Cardinality(DOMAIN messages) <= N");
            return 0;
        }
        return refuse("is not a state bound the engine implements (currentTerm[i] <= N, Len(log[i]) <= N, "
                      "Cardinality(DOMAIN messages) <= N, messages[m] <= N, conjoined)");
    };
    for (const auto& cn : C.constraints) {
        const Unit* d = X.def(cn);
        if (!d) return fail("CONSTRAINT " + cn + ": definition not found");
        std::vector<Tok> one{{cn, d->line, 1}};
        if (int rc = item(cn, *d, one, 0, 1, 0)) return fail(e), rc;
    }
    g.max_term = bd.term;
    g.max_log_len = bd.log;
    g.max_msgs = bd.msgs;
    g.max_dup = bd.dup;
    if (simulate) {  // unbounded fields: the wide layout's capacity (rmc_simulate truncates beyond it)
        if (g.max_term < 0) g.max_term = RMC_WIDE_MAX_TERM;
        if (g.max_log_len < 0) g.max_log_len = RMC_WIDE_MAX_LOG;
        if (g.max_msgs < 0) g.max_msgs = RMC_WIDE_MAX_MSGS;
        if (g.max_dup < 0) g.max_dup = RMC_WIDE_MAX_DUP;
    } else if (options & RMC_FRONT_DEPTH_BOUNDED) {
        // TLC -depth on a model that leaves fields unbounded (MCraft.cfg as
        // shipped): the wide layout's capacity, and a successor beyond it is an error
        if (g.max_term < 0) { g.max_term = RMC_WIDE_MAX_TERM; flags |= RMC_FLAG_UNBOUNDED_TERM; }
        if (g.max_log_len < 0) { g.max_log_len = RMC_WIDE_MAX_LOG; flags |= RMC_FLAG_UNBOUNDED_LOG; }
        if (g.max_msgs < 0) { g.max_msgs = RMC_WIDE_MAX_MSGS; flags |= RMC_FLAG_UNBOUNDED_MSGS; }
        if (g.max_dup < 0) { g.max_dup = RMC_WIDE_MAX_DUP; flags |= RMC_FLAG_UNBOUNDED_DUP; }
        if (flags & (RMC_FLAG_UNBOUNDED_TERM | RMC_FLAG_UNBOUNDED_LOG | RMC_FLAG_UNBOUNDED_MSGS | RMC_FLAG_UNBOUNDED_DUP))
            notes.push_back("no CONSTRAINT bounds every field: the search runs under the depth bound on the wide "
                            "layout and stops with a capacity error if a successor exceeds it (currentTerm 255, "
                            "Len(log) 32, 64 messages, count 255)");
    }
    if (g.max_term < 0 || g.max_log_len < 0 || g.max_msgs < 0 || g.max_dup < 0)
        return fail("the model is infinite without a CONSTRAINT bounding currentTerm, Len(log), "
                    "Cardinality(DOMAIN messages) and messages[m] (SURVEY.md §0.2); give a depth bound "
                    "(rmc-tlc -depth N, RMC_FRONT_DEPTH_BOUNDED) to explore it level by level");
    // ---- invariants
    static const struct { const char* name; uint32_t bit; } kInv[] = {
        {"OneLeaderPerTerm", RMC_INV_ONE_LEADER}, {"LogMatching", RMC_INV_LOG_MATCHING},
        {"MessagesInv", RMC_INV_MESSAGES}, {"LeaderVotesQuorum", RMC_INV_LEADER_VOTES},
        {"CandidateTermNotInLog", RMC_INV_CAND_TERM}, {"VotesGrantedInv", RMC_INV_VOTES_GRANTED},
        {"QuorumLogInv", RMC_INV_QUORUM_LOG}, {"MoreUpToDateCorrect", RMC_INV_MORE_UP_TO_DATE},
        {"LeaderCompleteness", RMC_INV_LEADER_COMPLETE}};
    for (const auto& in : C.invariants) {
        if (in == "TypeOK") {  // raft.tla:482-492 (checked with raft.tla above)
            g.invariants |= RMC_INV_TYPEOK;
            continue;
        }
        uint32_t bit = 0;
        for (const auto& k : kInv) if (in == k.name) bit = k.bit;
        if (!bit) return fail("INVARIANT " + in + " is not compiled into the engine");
        const Module* where = nullptr;
        if (!X.def(in, &where))
            return fail("INVARIANT " + in + " is not defined by the model (raft.tla's proof invariants sit past its "
                        "module end, raft.tla:505; define it as specs/MCraftBounded.tla does)");
        if (!known_def(in.c_str(), X.deep(in, {})))
            return fail("INVARIANT " + in + ": the definition in " + where->path +
                        " is not the one compiled into the engine (specs/MCraftBounded.tla)");
        g.invariants |= bit;
    }
    // ---- symmetry: exactly Permutations(<the Server set>)
    for (const auto& sy : C.symmetry) {
        const Unit* d = X.def(sy);
        if (!d) return fail("SYMMETRY " + sy + ": definition not found");
        const std::vector<Tok> bt = tokenize(*d, true);
        const bool perm = bt.size() == 4 && bt[0].t == "Permutations" && bt[1].t == "(" && bt[3].t == ")" &&
                          (bt[2].t == "Server" || (!server_set.empty() && bt[2].t == server_set));
        if (!perm)
            return fail("SYMMETRY " + sy + " is `" + join(bt, 0, bt.size()) +
                        "`; the engine implements only Permutations(Server)");
        flags |= RMC_FLAG_SYMMETRY;
    }
    if (C.check_deadlock == "FALSE") flags &= ~RMC_FLAG_CHECK_DEADLOCK;
    else if (!C.check_deadlock.empty() && C.check_deadlock != "TRUE")
        return fail("CHECK_DEADLOCK must be TRUE or FALSE");
    g.flags = flags;
    *out = g;
    if (info && info_cap) {
        std::string all;
        for (const auto& n : notes) all += (all.empty() ? "" : "\n") + n;
        snprintf(info, info_cap, "%s", all.c_str());
    }
    return 0;
}

static uint32_t env_options() {
    const char* b = getenv("RMC_BUILTIN_RAFT");
    return (b && b[0] == '1') ? RMC_FRONT_BUILTIN_RAFT : 0u;
}

extern "C" int rmc_model_from_files(const char* cfg_path, const char* tla_path, const char* raft_path,
                                    uint32_t options, rmc_config* cfg, rmc_sim_config* sim, char* info,
                                    size_t info_cap) {
    return parse_model(cfg_path, tla_path, raft_path, options, cfg, sim, info, info_cap);
}

extern "C" int rmc_config_from_files(const char* cfg_path, const char* tla_path, rmc_config* out, char* err,
                                     size_t err_cap) {
    return parse_model(cfg_path, tla_path, nullptr, env_options(), out, nullptr, err, err_cap);
}

extern "C" int rmc_sim_config_from_files(const char* cfg_path, const char* tla_path, rmc_config* out,
                                         rmc_sim_config* sim, char* err, size_t err_cap) {
    if (!sim) {
        if (err && err_cap) snprintf(err, err_cap, "null argument");
        return RMC_E_PARSE;
    }
    return parse_model(cfg_path, tla_path, nullptr, env_options() | RMC_FRONT_SIMULATE, out, sim, err, err_cap);
}

extern "C" int rmc_action_location(const char* action, int32_t* out4) {
    if (!action || !out4) return RMC_E_INVAL;
    for (const auto& s : kActionSpans)
        if (strcmp(s.action, action) == 0) {
            out4[0] = s.l1; out4[1] = s.c1; out4[2] = s.l2; out4[3] = s.c2;
            return 0;
        }
    return RMC_E_INVAL;
}
