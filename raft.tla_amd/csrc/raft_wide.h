// raft_wide.h — the wide state layout: raft.tla states beyond the packed capacity.
//
// The packed layout (raft_packed.h) holds terms <= 14 (15 for a successor
// that the CONSTRAINT rejects), logs of <= 3 entries, <= 8 distinct messages
// and counts <= 3: enough for every bounded model the BFS benchmarks, not for
// the reference's own configurations, which bound nothing — MCraft.cfg as
// shipped (terms grow at raft.tla:146-148, logs at :206-211, counts at
// :410-412) and Smokeraft.cfg's depth-100 walks (Smokeraft.cfg:46-48).  This
// layout is one byte per scalar field: terms and counts up to 255, logs of up
// to 32 entries, up to 64 distinct messages, and a canonical form in which
// byte equality is TLA+ value equality (fields a message type does not use
// are 0; the bag is sorted by the message bytes; unused entries and slots are
// 0).  The search on it is the same BFS (one lane per action instance, at most
// one successor per lane) without the packed layout's
// incremental tricks: a lane copies its parent, applies the action, and the
// fingerprint hashes the whole 5,080-byte record.  Models whose bounds fit the
// packed capacity never use it.
//
// Compiled for the host (codec) and for gfx950 (rmc_wide.hip).
#pragma once
#include <stdint.h>

#include "raft_packed.h"

namespace rmc {
namespace wide {

constexpr int WS = 5;    // servers held (= the packed layout's)
constexpr int LW = 32;   // log entries per server (rmc.h RMC_WIDE_MAX_LOG)
constexpr int KW = 64;   // distinct messages in the bag (rmc.h RMC_WIDE_MAX_MSGS)
// The compact record (DESIGN.md "Wide state"): 16 log entries and 16 messages,
// 904 bytes instead of 5,080 — enough for any state of a BFS bounded at depth
// 17 or less (each step adds at most one log entry and one distinct message)
// and for CONSTRAINTs of at most 16 entries and messages.
constexpr int LWC = 16, KWC = 16;
// The depth-sized record (round 6): 4 log entries and 12 messages, 336 bytes —
// enough for any state of a BFS bounded at depth 14 or less of a model whose
// logs and bag no CONSTRAINT bounds (MCraft.cfg as shipped).  Every log entry
// comes from a ClientRequest, which needs a leader: from Init (every server a
// term-1 follower) that takes at least Timeout(i), RequestVote(i, i) and
// RequestVote(i, j), the Receive of both requests, one UpdateTerm (or Timeout)
// of j to reach i's term, the Receive of both responses and BecomeLeader — 9
// steps for a quorum of 2 of 3 (5 with the weakened quorum of config 5: one
// granted vote) — and each later step adds at most one entry, so after n steps
// a log holds at most n - 9 (n - 5) entries.  The bag holds at most n - 1
// messages (the first step, Restart or Timeout, adds none).  A successor beyond
// the record is still caught (W_LOG / W_MSGS: a capacity error, never a silent cut).
constexpr int LWD = 4, KWD = 12;
constexpr int TMAX = 255, CMAX = 255;  // largest term / count a field holds
constexpr uint8_t NIL = 255;           // votedFor = Nil

struct WEnt {
    uint8_t term, value;
};
// One message record (raft.tla:443-475): 8 + 2 L bytes, fields a type does not use 0.
template <int L>
struct alignas(8) WMsgT {
    uint8_t type, term, src, dst;  // mtype, mterm, msource, mdest
    int8_t a;    // RVP mvoteGranted | AEQ mprevLogIndex (-1: Smokeraft.tla:35) | AEP msuccess
    uint8_t b;   // RVQ mlastLogTerm | AEQ mprevLogTerm | AEP mmatchIndex (unsigned: terms up to TMAX)
    uint8_t c;   // RVQ mlastLogIndex | AEQ mcommitIndex
    uint8_t n;   // AEQ Len(mentries) (<= 1) | RVP Len(mlog)
    WEnt e[L];   // AEQ mentries | RVP mlog (= log[i], raft.tla:259)
};
// The ten variables of raft.tla:31-74, with L log entries per server and K
// distinct messages (kLW / kKW: the record's capacity, Msg: its message type).
template <int L, int K>
struct WStateT {
    static constexpr int kLW = L, kKW = K;
    typedef WMsgT<L> Msg;
    uint8_t ct[WS], st[WS], vf[WS], ci[WS], len[WS], vR[WS], vG[WS];
    uint8_t nmsg;
    uint8_t ni[WS][WS], mi[WS][WS];
    uint8_t pad[2];
    WEnt log[WS][L];
    uint8_t cnt[K];
    Msg msg[K];
};
typedef WMsgT<LW> WMsg;
typedef WStateT<LW, KW> WState;     // the full record (5,080 B): simulation, rmc_expand, deep BFS
typedef WStateT<LWC, KWC> WStateC;  // the compact record (904 B): BFS of depth <= 17
typedef WStateT<LWD, KWD> WStateD;  // the depth-sized record (336 B): BFS of depth <= 14
static_assert(sizeof(WMsg) == 8 + 2 * LW && sizeof(WMsg) % 8 == 0, "WMsg layout");
static_assert(sizeof(WState) == 5080 && sizeof(WStateC) == 904 && sizeof(WStateD) == 336, "wide record sizes");
static_assert(sizeof(WState) % 8 == 0 && sizeof(WStateC) % 8 == 0 && sizeof(WStateD) % 8 == 0,
              "records are read as u64 words");
constexpr int WMWORDS = (int)(sizeof(WMsg) / 8);
constexpr int WWORDS = (int)(sizeof(WState) / 8);

// Lane table with KW message lanes per bag family; WLMASK u64
// words hold a mask over every lane of the largest shape (S = 5).
constexpr int WLANES_MAX = 5 + 5 + 25 + 5 + 5 * VMAX + 5 + 25 + 3 * KW;
constexpr int WLMASK = (WLANES_MAX + 63) / 64;
struct WLanes {
    int off[11];
    RMC_HD void init(int S) {
        const int n[10] = {S, S, S * S, S, S * VMAX, S, S * S, KW, KW, KW};
        off[0] = 0;
        for (int f = 0; f < 10; ++f) off[f + 1] = off[f] + n[f];
    }
    RMC_HD int family(int lane) const {
        int f = 0;
        while (f < 9 && lane >= off[f + 1]) ++f;
        return f;
    }
};

struct WModel {
    int S, V;
    int max_term, max_log, max_msgs, max_dup;  // CONSTRAINT bounds (<= the wide capacity)
    int unbounded;  // fields with no CONSTRAINT (1 term, 2 log, 4 msgs, 8 dup): beyond the
                    // wide capacity they are an error, not a filter
    int bug_quorum, inv_mask;
    WLanes L;
};

RMC_HD int wmemcmp(const void* a, const void* b, int n) {
    const uint8_t* x = (const uint8_t*)a;
    const uint8_t* y = (const uint8_t*)b;
    for (int k = 0; k < n; ++k)
        if (x[k] != y[k]) return x[k] < y[k] ? -1 : 1;
    return 0;
}
RMC_HD void wzero(void* p, int n) {
    uint8_t* x = (uint8_t*)p;
    for (int k = 0; k < n; ++k) x[k] = 0;
}
RMC_HD void wcopy(void* d, const void* s, int n) {
    uint8_t* x = (uint8_t*)d;
    const uint8_t* y = (const uint8_t*)s;
    for (int k = 0; k < n; ++k) x[k] = y[k];
}
template <class St>
RMC_HD void wcopy_state(St& d, const St& s) {
    u64* x = reinterpret_cast<u64*>(&d);
    const u64* y = reinterpret_cast<const u64*>(&s);
    for (int k = 0; k < (int)(sizeof(St) / 8); ++k) x[k] = y[k];
}

// Message order of the canonical bag: the record as WMWORDS u64 words compared in
// turn (a total order; byte equality = record equality).  Host and device sort by it.
template <class Mg>
RMC_HD int wmsg_cmp(const Mg& a, const Mg& b) {
    const u64* x = reinterpret_cast<const u64*>(&a);
    const u64* y = reinterpret_cast<const u64*>(&b);
    for (int k = 0; k < (int)(sizeof(Mg) / 8); ++k)
        if (x[k] != y[k]) return x[k] < y[k] ? -1 : 1;
    return 0;
}
template <class Mg>
RMC_HD void wmsg_zero(Mg& m) {
    u64* x = reinterpret_cast<u64*>(&m);
    for (int k = 0; k < (int)(sizeof(Mg) / 8); ++k) x[k] = 0;
}

RMC_HD int wquorum(const WModel& M, unsigned set) { return 2 * __builtin_popcount(set) > M.S; }  // raft.tla:81
template <class St>
RMC_HD int wlast_term(const St& s, int i) { return s.len[i] ? s.log[i][s.len[i] - 1].term : 0; }  // :84

template <class St>
RMC_HD void winit(const WModel& M, St& s) {  // Init raft.tla:113-129
    wzero(&s, (int)sizeof s);
    for (int i = 0; i < M.S; ++i) {
        s.ct[i] = 1;
        s.st[i] = FOLLOWER;
        s.vf[i] = NIL;
        for (int j = 0; j < M.S; ++j) s.ni[i][j] = 1;
    }
}

// Lane results: not enabled, enabled (the successor is in t), or enabled with a
// successor the wide layout cannot hold — the field it overflows (an error
// for fields no CONSTRAINT bounds; the packed layout's capacity bits).
enum : int { W_OFF = 0, W_ON = 1, W_TERM = 2, W_LOG = 3, W_MSGS = 4, W_DUP = 5 };
RMC_HD int woverflow_bits(int code) { return code >= W_TERM ? 1 << (code - W_TERM) : 0; }

// Would Bag (+) SetToBag({m}) fit (without changing s)?
template <class St>
RMC_HD int wbag_fits(const St& s, const typename St::Msg& m) {
    for (int k = 0; k < s.nmsg; ++k)
        if (wmsg_cmp(s.msg[k], m) == 0) return s.cnt[k] >= CMAX ? W_DUP : W_ON;
    return s.nmsg >= St::kKW ? W_MSGS : W_ON;
}
// Would Reply(r, s.msg[x]) (raft.tla:102-103: add the response, remove the
// request) fit?  The capacity is that of the resulting bag: a request with count
// 1 frees its slot (r never equals a request: the types differ).
template <class St>
RMC_HD int wreply_fits(const St& s, const typename St::Msg& r, int x) {
    for (int k = 0; k < s.nmsg; ++k)
        if (wmsg_cmp(s.msg[k], r) == 0) return s.cnt[k] >= CMAX ? W_DUP : W_ON;
    return (s.nmsg >= St::kKW && s.cnt[x] > 1) ? W_MSGS : W_ON;
}
// Bag (+) SetToBag({m}) (raft.tla:88), kept sorted (call after wbag_fits).
template <class St>
RMC_HD int wbag_add(St& s, const typename St::Msg& m) {
    int k = 0;
    for (; k < s.nmsg; ++k) {
        const int c = wmsg_cmp(s.msg[k], m);
        if (c == 0) {
            if (s.cnt[k] >= CMAX) return W_DUP;
            s.cnt[k] += 1;
            return W_ON;
        }
        if (c > 0) break;
    }
    if (s.nmsg >= St::kKW) return W_MSGS;
    for (int q = s.nmsg; q > k; --q) {
        s.msg[q] = s.msg[q - 1];
        s.cnt[q] = s.cnt[q - 1];
    }
    s.msg[k] = m;
    s.cnt[k] = 1;
    s.nmsg += 1;
    return W_ON;
}
// Bag (-) SetToBag({m}) (raft.tla:92) of the message in slot k: a count that
// reaches 0 removes the key (Bags' (-)).
template <class St>
RMC_HD void wbag_remove_at(St& s, int k) {
    if (--s.cnt[k]) return;
    for (int q = k; q + 1 < s.nmsg; ++q) {
        s.msg[q] = s.msg[q + 1];
        s.cnt[q] = s.cnt[q + 1];
    }
    s.nmsg -= 1;
    wmsg_zero(s.msg[s.nmsg]);
    s.cnt[s.nmsg] = 0;
}

// The bag operations a lane applies: one thread at a time (SerialBag), or the
// whole wave on a record in LDS (WaveBag, rmc_wide.hip: every lane calls with
// the same arguments, each compares / moves one message).
struct SerialBag {
    template <class St>
    static RMC_HD int fits(const St& s, const typename St::Msg& m) { return wbag_fits(s, m); }
    template <class St>
    static RMC_HD int reply_fits(const St& s, const typename St::Msg& r, int x) { return wreply_fits(s, r, x); }
    template <class St>
    static RMC_HD int add(St& s, const typename St::Msg& m) { return wbag_add(s, m); }
    template <class St>
    static RMC_HD void remove_at(St& s, int k) { wbag_remove_at(s, k); }
};

// Lane `lane` on s (raft.tla:136-417, one action instance): W_OFF when the
// instance is not enabled, W_ON when it is (*t = the successor, if t is
// given), else the field its successor overflows (W_TERM .. W_DUP; *t is not
// written).  t == nullptr only evaluates the guard (the simulation's draw): W_OFF
// or not — a nonzero code may then be W_ON for a successor that would not fit,
// which the draw treats alike (it is decided when the drawn lane is applied);
// pre: *t already holds a copy of s (a wave that copied it cooperatively), or
// t == &s (every field of s is read before the same field of *t is written).
// Scalar fields of *t are written from s (never read-modify-written), so a
// wave whose lanes all apply the same lane to a shared record writes the same
// values.
template <class T>
struct WSame {  // a non-deduced parameter type (t may be nullptr)
    typedef T type;
};
// What a lane changed (the BFS's incremental fingerprint, wfp_delta): the
// server whose fields it may have written, the message of s it removed one copy
// of or duplicated (slot in s), and the slot in t of the message it added.
struct WDelta {
    int srv, rm, dup, add_at;
};
template <class St>
RMC_HD int wfind(const St& t, const typename St::Msg& m) {
    for (int k = 0; k < t.nmsg; ++k)
        if (wmsg_cmp(t.msg[k], m) == 0) return k;
    return -1;
}
template <class Bag = SerialBag, class St = WState>
RMC_HD int wlane(const WModel& M, const St& s, int lane, typename WSame<St>::type* t, bool pre = false,
                 WDelta* dl = nullptr) {
    typedef typename St::Msg WMsg;
    constexpr int LW = St::kLW;
    const int S = M.S;
    const int f = M.L.family(lane), x = lane - M.L.off[f];
    if (dl) *dl = WDelta{f <= 5 ? (f == 2 ? -1 : f == 4 ? x / VMAX : x) : -1, -1, -1, -1};
    switch (f) {
    case 0: {  // Restart(i) :136-143 — always enabled
        const int i = x;
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        t->st[i] = FOLLOWER;
        t->vR[i] = 0;
        t->vG[i] = 0;
        t->ci[i] = 0;
        for (int j = 0; j < S; ++j) {
            t->ni[i][j] = 1;
            t->mi[i][j] = 0;
        }
        return W_ON;
    }
    case 1: {  // Timeout(i) :146-154
        const int i = x;
        if (s.st[i] != FOLLOWER && s.st[i] != CANDIDATE) return W_OFF;
        if (s.ct[i] >= TMAX) return W_TERM;
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        t->st[i] = CANDIDATE;
        t->ct[i] = (uint8_t)(s.ct[i] + 1);
        t->vf[i] = NIL;
        t->vR[i] = 0;
        t->vG[i] = 0;
        return W_ON;
    }
    case 2: {  // RequestVote(i, j) :157-166 (no i /= j guard)
        const int i = x / S, j = x % S;
        if (s.st[i] != CANDIDATE || ((s.vR[i] >> j) & 1u)) return W_OFF;
        if (!t) return W_ON;
        WMsg m;
        wmsg_zero(m);
        m.type = RVQ;
        m.term = s.ct[i];
        m.b = (uint8_t)wlast_term(s, i);
        m.c = s.len[i];
        m.src = (uint8_t)i;
        m.dst = (uint8_t)j;
        const int fit = Bag::fits(s, m);
        if (fit != W_ON) return fit;
        if (!pre) wcopy_state(*t, s);
        const int r = Bag::add(*t, m);
        if (dl) dl->add_at = wfind(*t, m);
        return r;
    }
    case 3: {  // BecomeLeader(i) :195-203
        const int i = x;
        if (s.st[i] != CANDIDATE) return W_OFF;
        if (M.bug_quorum ? s.vG[i] == 0 : !wquorum(M, s.vG[i])) return W_OFF;
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        t->st[i] = LEADER;
        for (int j = 0; j < S; ++j) {
            t->ni[i][j] = (uint8_t)(s.len[i] + 1);
            t->mi[i][j] = 0;
        }
        return W_ON;
    }
    case 4: {  // ClientRequest(i, v) :206-213
        const int i = x / VMAX, v = x % VMAX;
        if (v >= M.V || s.st[i] != LEADER) return W_OFF;
        if (s.len[i] >= LW) return W_LOG;
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        t->log[i][s.len[i]].term = s.ct[i];
        t->log[i][s.len[i]].value = (uint8_t)v;
        t->len[i] = (uint8_t)(s.len[i] + 1);
        return W_ON;
    }
    case 5: {  // AdvanceCommitIndex(i) :219-236
        const int i = x;
        if (s.st[i] != LEADER) return W_OFF;
        if (!t) return W_ON;
        int best = 0;
        for (int idx = 1; idx <= s.len[i]; ++idx) {
            unsigned agree = 1u << i;
            for (int q = 0; q < S; ++q)
                if (s.mi[i][q] >= idx) agree |= 1u << q;
            if (wquorum(M, agree)) best = idx;  // Max(agreeIndexes)
        }
        if (!pre) wcopy_state(*t, s);
        if (best > 0 && s.log[i][best - 1].term == s.ct[i]) t->ci[i] = (uint8_t)best;
        return W_ON;
    }
    case 6: {  // AppendEntries(i, j) :171-192
        const int i = x / S, j = x % S;
        if (i == j || s.st[i] != LEADER) return W_OFF;
        if (!t) return W_ON;
        const int nidx = s.ni[i][j], len = s.len[i];
        const int prev = nidx - 1;
        const int last = len < nidx ? len : nidx;  // Min({Len(log[i]), nextIndex[i][j]})
        WMsg m;
        wmsg_zero(m);
        m.type = AEQ;
        m.term = s.ct[i];
        m.a = (int8_t)prev;
        m.b = (uint8_t)((prev > 0 && prev <= len) ? s.log[i][prev - 1].term : 0);
        if (nidx <= last) {  // SubSeq(log[i], nextIndex, last): 0 or 1 entry
            m.n = 1;
            m.e[0] = s.log[i][nidx - 1];
        }
        m.c = (uint8_t)(s.ci[i] < last ? s.ci[i] : last);
        m.src = (uint8_t)i;
        m.dst = (uint8_t)j;
        const int fit = Bag::fits(s, m);
        if (fit != W_ON) return fit;
        if (!pre) wcopy_state(*t, s);
        const int r = Bag::add(*t, m);
        if (dl) dl->add_at = wfind(*t, m);
        return r;
    }
    case 7: {  // Receive(m) :388-403 for bag slot x
        if (x >= s.nmsg) return W_OFF;
        const WMsg& m = s.msg[x];
        const int i = m.dst, j = m.src, ct = s.ct[i];
        if (dl) dl->srv = i;  // (a branch that leaves m in the bag: only the server changes)
        if (m.term > ct) {  // UpdateTerm :373-379 — m stays
            if (!t) return W_ON;
            if (!pre) wcopy_state(*t, s);
            t->ct[i] = m.term;
            t->st[i] = FOLLOWER;
            t->vf[i] = NIL;
            return W_ON;
        }
        if (m.type == RVQ) {  // HandleRequestVoteRequest :244-263
            if (!t) return W_ON;
            const int lt = wlast_term(s, i);
            const int logok = m.b > lt || (m.b == lt && m.c >= s.len[i]);
            const int grant = m.term == ct && logok && (s.vf[i] == NIL || s.vf[i] == j);
            WMsg r;
            wmsg_zero(r);
            r.type = RVP;
            r.term = (uint8_t)ct;
            r.src = (uint8_t)i;
            r.dst = (uint8_t)j;
            r.a = (int8_t)grant;
            r.n = s.len[i];
            for (int e = 0; e < s.len[i]; ++e) r.e[e] = s.log[i][e];
            // Reply :102-103 (response added, request removed): the capacity of the net bag
            const int fit = Bag::reply_fits(s, r, x);
            if (fit != W_ON) return fit;
            if (!pre) wcopy_state(*t, s);
            if (grant) t->vf[i] = (uint8_t)j;
            Bag::remove_at(*t, x);
            Bag::add(*t, r);
            if (dl) {
                dl->rm = x;
                dl->add_at = wfind(*t, r);
            }
            return W_ON;
        }
        if (m.type == RVP) {
            if (!t) return W_ON;
            if (!pre) wcopy_state(*t, s);
            if (m.term == ct) {  // HandleRequestVoteResponse :267-279
                t->vR[i] = (uint8_t)(s.vR[i] | (1u << j));
                if (m.a) t->vG[i] = (uint8_t)(s.vG[i] | (1u << j));
            }  // else DropStaleResponse :382-385
            Bag::remove_at(*t, x);
            if (dl) dl->rm = x;
            return W_ON;
        }
        if (m.type == AEQ) {  // HandleAppendEntriesRequest :347-356
            const int pidx = m.a;
            const int logok = pidx == 0 || (pidx > 0 && pidx <= s.len[i] && m.b == s.log[i][pidx - 1].term);
            WMsg r;
            wmsg_zero(r);
            r.type = AEP;
            r.term = (uint8_t)ct;
            r.src = (uint8_t)i;
            r.dst = (uint8_t)j;
            if (m.term < ct || (s.st[i] == FOLLOWER && !logok)) {  // Reject :281-293
                if (!t) return W_ON;
                const int fit = Bag::reply_fits(s, r, x);
                if (fit != W_ON) return fit;
                if (!pre) wcopy_state(*t, s);
                Bag::remove_at(*t, x);
                Bag::add(*t, r);
                if (dl) {
                    dl->rm = x;
                    dl->add_at = wfind(*t, r);
                }
                return W_ON;
            }
            if (s.st[i] == CANDIDATE) {  // ReturnToFollowerState :295-299 — m stays
                if (!t) return W_ON;
                if (!pre) wcopy_state(*t, s);
                t->st[i] = FOLLOWER;
                return W_ON;
            }
            if (s.st[i] != FOLLOWER) return W_OFF;  // a Leader: no branch is enabled
            const int index = pidx + 1, len = s.len[i];
            if (m.n == 0 || (len >= index && s.log[i][index - 1].term == m.e[0].term)) {
                // AppendEntriesAlreadyDone :301-317: UNCHANGED logVars after binding
                // commitIndex' is an equality test under TLC
                if (m.c != s.ci[i]) return W_OFF;
                if (!t) return W_ON;
                r.a = 1;
                r.b = (uint8_t)(pidx + m.n);
                const int fit = Bag::reply_fits(s, r, x);
                if (fit != W_ON) return fit;
                if (!pre) wcopy_state(*t, s);
                Bag::remove_at(*t, x);
                Bag::add(*t, r);
                if (dl) {
                    dl->rm = x;
                    dl->add_at = wfind(*t, r);
                }
                return W_ON;
            }
            if (len >= index) {  // ConflictAppendEntriesRequest :319-325 — drops the LAST entry, m stays
                if (!t) return W_ON;
                if (!pre) wcopy_state(*t, s);
                t->len[i] = (uint8_t)(len - 1);
                t->log[i][len - 1].term = 0;
                t->log[i][len - 1].value = 0;
                return W_ON;
            }
            if (len == pidx) {  // NoConflictAppendEntriesRequest :327-331 — m stays
                if (len >= LW) return W_LOG;
                if (!t) return W_ON;
                if (!pre) wcopy_state(*t, s);
                t->log[i][len] = m.e[0];
                t->len[i] = (uint8_t)(len + 1);
                return W_ON;
            }
            return W_OFF;
        }
        // AEP
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        if (m.term == ct) {  // HandleAppendEntriesResponse :360-370 (no Leader guard)
            if (m.a) {
                t->ni[i][j] = (uint8_t)(m.b + 1);
                t->mi[i][j] = m.b;
            } else {
                const int v = s.ni[i][j] - 1;
                t->ni[i][j] = (uint8_t)(v < 1 ? 1 : v);
            }
        }  // else DropStaleResponse
        Bag::remove_at(*t, x);
        if (dl) dl->rm = x;
        return W_ON;
    }
    case 8: {  // DuplicateMessage(m) :410-412
        if (x >= s.nmsg) return W_OFF;
        if (s.cnt[x] >= CMAX) return W_DUP;
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        t->cnt[x] = (uint8_t)(s.cnt[x] + 1);
        if (dl) dl->dup = x;
        return W_ON;
    }
    default: {  // DropMessage(m) :415-417
        if (x >= s.nmsg) return W_OFF;
        if (!t) return W_ON;
        if (!pre) wcopy_state(*t, s);
        Bag::remove_at(*t, x);
        if (dl) dl->rm = x;
        return W_ON;
    }
    }
}

// CONSTRAINT of a successor the layout holds: 1 in the model, 0 filtered
// (generated, neither stored nor checked).
template <class St>
RMC_HD int win_model(const WModel& M, const St& t) {
    int ok = 1;
    for (int i = 0; i < M.S; ++i) {
        if (t.ct[i] > M.max_term) ok = 0;
        if (t.len[i] > M.max_log) ok = 0;
    }
    if (t.nmsg > M.max_msgs) ok = 0;
    for (int q = 0; q < t.nmsg; ++q)
        if (t.cnt[q] > M.max_dup) ok = 0;
    return ok;
}

// ---- invariants (raft.tla:482-492; the config-5 and proof invariants as restated
// in specs/MCraftBounded.tla) --------------------------------------------------------
template <class St>
RMC_HD int wtype_ok(const WModel& M, const St& s) {  // raft.tla:482-492
    for (int i = 0; i < M.S; ++i) {
        if (s.st[i] > LEADER) return 0;
        if (s.vf[i] != NIL && s.vf[i] >= M.S) return 0;
        if ((s.vR[i] | s.vG[i]) >> M.S) return 0;
        for (int j = 0; j < M.S; ++j)
            if (s.ni[i][j] < 1) return 0;
        for (int x = 0; x < s.len[i]; ++x)
            if (s.log[i][x].value >= M.V) return 0;
    }
    for (int q = 0; q < s.nmsg; ++q) {
        const auto& m = s.msg[q];
        if (s.cnt[q] < 1 || m.src >= M.S || m.dst >= M.S) return 0;
        for (int x = 0; x < m.n; ++x)
            if (m.e[x].value >= M.V) return 0;
    }
    return 1;
}
template <class St>
RMC_HD int wcommitted_prefix_of(const St& s, int j, int i) {  // IsPrefix(Committed(j), log[i])
    const int c = s.ci[j] < s.len[j] ? s.ci[j] : s.len[j];
    if (s.len[i] < c) return 0;
    return wmemcmp(s.log[i], s.log[j], c * (int)sizeof(WEnt)) == 0;
}
// 0 = every named invariant holds, else the RMC_INV_* bit (index) of the first violated one + 1
template <class St>
RMC_HD int wcheck_invariants(const WModel& M, const St& s) {
    const int S = M.S, mask = M.inv_mask;
    if ((mask & 1) && !wtype_ok(M, s)) return 1;
    if (mask & 2)  // OneLeaderPerTerm (ElectionSafety restated, raft.tla:1124)
        for (int i = 0; i < S; ++i)
            for (int j = i + 1; j < S; ++j)
                if (s.st[i] == LEADER && s.st[j] == LEADER && s.ct[i] == s.ct[j]) return 2;
    if (mask & 4)  // LogMatching raft.tla:1132-1136
        for (int i = 0; i < S; ++i)
            for (int j = 0; j < S; ++j) {
                const int n = s.len[i] < s.len[j] ? s.len[i] : s.len[j];
                for (int x = 1; x <= n; ++x)
                    if (s.log[i][x - 1].term == s.log[j][x - 1].term &&
                        wmemcmp(s.log[i], s.log[j], x * (int)sizeof(WEnt)) != 0)
                        return 3;
            }
    if (mask & 8)  // MessagesInv raft.tla:941-946 (:910's m.dest read as m.mdest)
        for (int q = 0; q < s.nmsg; ++q) {
            const auto& m = s.msg[q];
            const int src = m.src, dst = m.dst, cs = s.ct[src];
            if (m.term > cs) return 4;  // :934-935
            if (m.type == RVP && m.a && cs == s.ct[dst] && cs == m.term) {  // :903-910
                const int ld = wlast_term(s, dst), ls = wlast_term(s, src);
                if (!(ld > ls || (ld == ls && s.len[dst] >= s.len[src]))) return 4;
            }
            if (m.type == RVQ && s.st[src] == CANDIDATE && cs == m.term)  // :915-920
                if (m.c != s.len[src] || m.b != wlast_term(s, src)) return 4;
            if (m.type == AEQ && m.n > 0 && m.term == cs) {  // :924-930
                const int p = m.a;
                if (p + 1 < 1 || p + 1 > s.len[src]) return 4;
                if (s.log[src][p].term != m.e[0].term || s.log[src][p].value != m.e[0].value) return 4;
                if (p > 0 && p <= s.len[src] && s.log[src][p - 1].term != m.b) return 4;
            }
        }
    if (mask & 16)  // LeaderVotesQuorum raft.tla:1033-1037
        for (int i = 0; i < S; ++i) {
            if (s.st[i] != LEADER) continue;
            unsigned q = 0;
            for (int j = 0; j < S; ++j)
                if (s.ct[j] > s.ct[i] || (s.ct[j] == s.ct[i] && s.vf[j] == i)) q |= 1u << j;
            if (!wquorum(M, q)) return 5;
        }
    if (mask & 32)  // CandidateTermNotInLog raft.tla:1041-1047
        for (int i = 0; i < S; ++i) {
            if (s.st[i] != CANDIDATE) continue;
            unsigned q = 0;
            for (int j = 0; j < S; ++j)
                if (s.ct[j] == s.ct[i] && (s.vf[j] == i || s.vf[j] == NIL)) q |= 1u << j;
            if (!wquorum(M, q)) continue;
            for (int j = 0; j < S; ++j)
                for (int n = 0; n < s.len[j]; ++n)
                    if (s.log[j][n].term == s.ct[i]) return 6;
        }
    if (mask & 64)  // VotesGrantedInv raft.tla:1145-1153
        for (int i = 0; i < S; ++i)
            for (int j = 0; j < S; ++j)
                if (((s.vG[i] >> j) & 1u) && s.ct[i] == s.ct[j] && !wcommitted_prefix_of(s, j, i)) return 7;
    if (mask & 128)  // QuorumLogInv raft.tla:1157-1161
        for (int i = 0; i < S; ++i) {
            unsigned miss = 0;
            for (int j = 0; j < S; ++j)
                if (!wcommitted_prefix_of(s, i, j)) miss |= 1u << j;
            if (wquorum(M, miss)) return 8;
        }
    if (mask & 256)  // MoreUpToDateCorrect raft.tla:1167-1172
        for (int i = 0; i < S; ++i)
            for (int j = 0; j < S; ++j) {
                const int li = wlast_term(s, i), lj = wlast_term(s, j);
                if ((li > lj || (li == lj && s.len[i] >= s.len[j])) && !wcommitted_prefix_of(s, j, i)) return 9;
            }
    if (mask & 512)  // LeaderCompleteness raft.tla:1176-1180
        for (int i = 0; i < S; ++i) {
            if (s.st[i] != LEADER) continue;
            for (int j = 0; j < S; ++j)
                if (!wcommitted_prefix_of(s, j, i)) return 10;
        }
    return 0;
}

RMC_HD u64 w_rand(u64& x) {  // splitmix64 stream (the simulators' draws)
    x += 0x9E3779B97F4A7C15ull;
    return mix64(x);
}

// TLC's simulator draw (tlc2.tool.Simulator, restated): Next's actions in
// order — every instance of Restart .. AppendEntries (TLC splits \E over the
// constant Server / Value sets into separate actions) and Receive,
// DuplicateMessage, DropMessage as one action each (their \E m \in DOMAIN
// messages ranges over the state) — are visited from a uniformly random start
// index with a random prime stride; the first action with a successor is taken
// and one of its successors drawn uniformly.  The strides are primes larger
// than any action count (at most 83 actions), so every stride visits every
// action.  en: the enabled lanes (bit l of en[l >> 6]); returns the lane, -1
// if none is enabled.
// Lanes [lo, hi) of the mask words: how many are set, and the k-th set one.
template <int NC>
RMC_HD u64 range_word(const u64 (&en)[NC], int c, int lo, int hi) {
    const int b0 = 64 * c;
    if (hi <= b0 || lo >= b0 + 64) return 0;
    u64 m = en[c];
    if (lo > b0) m &= ~0ull << (lo - b0);
    if (hi < b0 + 64) m &= (1ull << (hi - b0)) - 1ull;
    return m;
}
template <int NC>
RMC_HD int tlc_draw(const u64 (&en)[NC], int nl, int o7, int o8, int o9, u64& rs) {
    auto on = [&](int lane) { return ((en[lane >> 6] >> (lane & 63)) & 1ull) != 0; };
    const int nact = o7 + 3;
    const u32 primes[8] = {89, 97, 101, 103, 107, 109, 113, 127};
    const u32 start = (u32)(w_rand(rs) % (u64)nact), stride = primes[w_rand(rs) & 7u];
    const u32 step = stride % (u32)nact;  // (start + i * stride) % nact, one addition per action
    u32 a = start;
    for (int i = 0; i < nact; ++i, a = a + step >= (u32)nact ? a + step - (u32)nact : a + step) {
        if ((int)a < o7) {
            if (on((int)a)) return (int)a;
            continue;
        }
        const int f = (int)a - o7, lo = f == 0 ? o7 : f == 1 ? o8 : o9, hi = f == 0 ? o8 : f == 1 ? o9 : nl;
        u32 cnt = 0;
        for (int c = 0; c < NC; ++c) cnt += (u32)__builtin_popcountll(range_word<NC>(en, c, lo, hi));
        if (!cnt) continue;
        u32 k = (u32)(w_rand(rs) % (u64)cnt);  // the k-th enabled lane of the family, in lane order
        for (int c = 0; c < NC; ++c) {
            u64 m = range_word<NC>(en, c, lo, hi);
            const u32 p = (u32)__builtin_popcountll(m);
            if (k < p) {
                for (; k; --k) m &= m - 1;
                return 64 * c + __builtin_ctzll(m);
            }
            k -= p;
        }
    }
    return -1;
}

// The uniform draws (RMC_SIM_WITHIN_CAPACITY / RMC_SIM_TRUNCATE): one of the
// enabled lanes not excluded, uniformly, with one random number.
template <int NC>
RMC_HD int uniform_draw(const u64 (&en)[NC], const u64 (&excl)[NC], u64& rs) {
    u32 cnt = 0;
    for (int c = 0; c < NC; ++c) cnt += (u32)__builtin_popcountll(en[c] & ~excl[c]);
    if (!cnt) return -1;
    u32 k = (u32)(w_rand(rs) % (u64)cnt);
    for (int c = 0; c < NC; ++c) {
        u64 mm = en[c] & ~excl[c];
        const u32 p = (u32)__builtin_popcountll(mm);
        if (k < p) {
            for (; k; --k) mm &= mm - 1;
            return 64 * c + __builtin_ctzll(mm);
        }
        k -= p;
    }
    return -1;
}

// Fingerprint of a canonical record (salted like the packed one), round 6: like
// the packed layout's, an order-free sum over components — each server's fields
// (its log up to its length) and each message with its count, every component
// a short chained mix of its own bytes — so a successor's fingerprint is its
// parent's minus the components a lane changed plus their new values
// (wfp_delta: about 10 mixes instead of the whole record's 62-635 words).
// k = sum of the components mod 2^64, s = sum of their smix (raft_packed.h Fp).
// Unused log entries and message fields are 0 in the canonical form, so the
// record's capacity does not enter.
template <class St>
RMC_HD u64 wcomp_srv(const St& s, int i, u64 salt) {
    u64 w0 = (u64)s.ct[i] | ((u64)s.st[i] << 8) | ((u64)s.vf[i] << 16) | ((u64)s.ci[i] << 24) |
             ((u64)s.len[i] << 32) | ((u64)s.vR[i] << 40) | ((u64)s.vG[i] << 48) | ((u64)i << 56);
    u64 w1 = 0, w2 = 0;
    for (int j = 0; j < WS; ++j) {
        w1 |= (u64)s.ni[i][j] << (8 * j);
        w2 |= (u64)s.mi[i][j] << (8 * j);
    }
    u64 h = mix64(w0 ^ salt ^ 0x243F6A8885A308D3ull);
    h = mix64(h ^ w1 ^ (w2 << 40));
    h = mix64(h ^ (w2 >> 24));
    const int n = s.len[i];
    for (int e = 0; e < n; e += 4) {  // 4 entries (8 bytes) per word
        u64 lw = 0;
        for (int q = 0; q < 4 && e + q < n; ++q)
            lw |= ((u64)s.log[i][e + q].term | ((u64)s.log[i][e + q].value << 8)) << (16 * q);
        h = mix64(h ^ lw ^ ((u64)e << 58));
    }
    return h;
}
template <class Mg>
RMC_HD u64 wcomp_msg(const Mg& m, int cnt, u64 salt) {
    const u64 hdr = (u64)m.type | ((u64)m.term << 8) | ((u64)m.src << 16) | ((u64)m.dst << 24) |
                    ((u64)(uint8_t)m.a << 32) | ((u64)m.b << 40) | ((u64)m.c << 48) | ((u64)m.n << 56);
    u64 h = mix64(hdr ^ salt ^ 0x13198A2E03707344ull);
    h = mix64(h ^ (u64)(unsigned)cnt ^ 0xA4093822299F31D0ull);
    const int n = m.n;
    for (int e = 0; e < n; e += 4) {
        u64 lw = 0;
        for (int q = 0; q < 4 && e + q < n; ++q)
            lw |= ((u64)m.e[e + q].term | ((u64)m.e[e + q].value << 8)) << (16 * q);
        h = mix64(h ^ lw ^ ((u64)e << 58));
    }
    return h;
}
template <class St>
RMC_HD Fp wfp(const St& s, u64 salt, int S = WS) {
    Fp h{0, 0};
    for (int i = 0; i < S; ++i) fp_add(h, wcomp_srv(s, i, salt));
    for (int q = 0; q < s.nmsg; ++q) fp_add(h, wcomp_msg(s.msg[q], s.cnt[q], salt));
    return h;
}
// The successor t = lane(s) from s's fingerprint h0 and what the lane changed.
template <class St>
RMC_HD Fp wfp_delta(const St& s, const St& t, const Fp& h0, const WDelta& d, u64 salt) {
    Fp h = h0;
    if (d.srv >= 0) {
        fp_sub(h, wcomp_srv(s, d.srv, salt));
        fp_add(h, wcomp_srv(t, d.srv, salt));
    }
    if (d.rm >= 0) {
        const int c = s.cnt[d.rm];
        fp_sub(h, wcomp_msg(s.msg[d.rm], c, salt));
        if (c > 1) fp_add(h, wcomp_msg(s.msg[d.rm], c - 1, salt));
    }
    if (d.dup >= 0) {
        const int c = s.cnt[d.dup];
        fp_sub(h, wcomp_msg(s.msg[d.dup], c, salt));
        fp_add(h, wcomp_msg(s.msg[d.dup], c + 1, salt));
    }
    if (d.add_at >= 0) {
        const int c = t.cnt[d.add_at];
        fp_add(h, wcomp_msg(t.msg[d.add_at], c, salt));
        if (c > 1) fp_sub(h, wcomp_msg(t.msg[d.add_at], c - 1, salt));
    }
    return h;
}

}  // namespace wide
}  // namespace rmc
