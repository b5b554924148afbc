/*
 * rmc_oracle.c — CPU restatement of raft.tla + TLC's BFS loop.
 *
 * TEST INFRASTRUCTURE ONLY (the oracle and the CPU baseline "port").  The
 * product engine lives in raft.tla_amd/ and never links this file.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may run it.
 *
 * It is an independent second restatement of raft.tla:81-434 (the first is
 * oracle/raft_spec.py): plain C structs with one field per TLA+ variable,
 * messages kept as a sorted array of (record, count) pairs, and an EXACT
 * full-state hash set (no fingerprints), so its distinct-state counts carry
 * no collision risk.  Every action cites the raft.tla lines it follows.
 *
 * TLC semantics restated:
 *   - AppendEntriesAlreadyDone (raft.tla:301-317) is enabled only when
 *     m.mcommitIndex = commitIndex[i] (UNCHANGED logVars after binding
 *     commitIndex' is an equality test under TLC);
 *   - Bags (-) drops a key whose count reaches 0 (raft.tla:92);
 *   - CONSTRAINT is applied before the seen-set; out-of-constraint
 *     successors count as generated but are neither stored nor checked;
 *   - "generated" = initial states + every successor of every expanded state.
 *
 * Build: see oracle/Makefile (gcc -O2 -pthread).  Interfaces:
 *   CLI:   rmc_oracle S V MaxTerm MaxLog MaxMsgs MaxDup [threads] [max_levels]
 *                      [bug_quorum] [inv_mask] [symmetry] [capacity]
 *   C ABI: orc_bfs(...) for ctypes (tests / bench cpu_baseline).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define OS 5  /* max servers */
#ifndef OL
#define OL 4  /* max log length held (bounds are <= 3, +1 overshoot); liboracle_wide.so: 9 */
#endif
#ifndef OK_
#define OK_ 9 /* max distinct messages held (bounds are <= 8, +1 overshoot); liboracle_wide.so: 13 */
#endif

enum { FOLLOWER = 0, CANDIDATE = 1, LEADER = 2 };
enum { NIL = 15 };
enum { RVQ = 0, RVP = 1, AEQ = 2, AEP = 3 }; /* raft.tla:23-24 */

typedef struct { int8_t term, value; } ent_t;

/* One message record.  Unused fields are zero so memcmp is record equality. */
typedef struct {
    int8_t type, term, src, dst;
    int8_t a;      /* RVQ: mlastLogTerm  AEQ: mprevLogIndex  RVP: mvoteGranted  AEP: msuccess */
    int8_t b;      /* RVQ: mlastLogIndex AEQ: mprevLogTerm                    AEP: mmatchIndex */
    int8_t c;      /* AEQ: mcommitIndex */
    int8_t n;      /* AEQ: Len(mentries)  RVP: Len(mlog) */
    ent_t e[OL];   /* AEQ: mentries       RVP: mlog */
} msg_t;

typedef struct {
    int8_t ct[OS], st[OS], vf[OS], ci[OS], len[OS];
    ent_t log[OS][OL];
    uint8_t vR[OS], vG[OS];
    int8_t ni[OS][OS], mi[OS][OS];
    int8_t nmsg, pad[3];
    msg_t msg[OK_];
    uint8_t cnt[OK_];
    uint8_t pad2[7];
} ost_t;

typedef struct {
    int S, V, max_term, max_log, max_msgs, max_dup, bug_quorum, inv_mask, symmetry;
} omodel_t;

#define INV_TYPEOK 1
#define INV_ONE_LEADER 2
#define INV_LOG_MATCHING 4
#define INV_MESSAGES 8
#define INV_LEADER_VOTES 16
#define INV_CAND_TERM 32
#define INV_VOTES_GRANTED 64
#define INV_QUORUM_LOG 128
#define INV_MORE_UP_TO_DATE 256
#define INV_LEADER_COMPLETE 512

/* ---------------- helpers (raft.tla:81-108) ---------------- */
static int popc(unsigned x) { return __builtin_popcount(x); }
static int is_quorum(const omodel_t* M, unsigned set) { return popc(set) * 2 > M->S; } /* :81 */
static int last_term(const ost_t* s, int i) { return s->len[i] ? s->log[i][s->len[i] - 1].term : 0; } /* :84 */

static int msg_cmp(const msg_t* a, const msg_t* b) { return memcmp(a, b, sizeof(msg_t)); }

/* WithMessage (:88): bag (+) SetToBag({m}); returns 0 if the held capacity overflows. */
static int bag_add(ost_t* s, const msg_t* m) {
    int k;
    for (k = 0; k < s->nmsg; k++) {
        int c = msg_cmp(&s->msg[k], m);
        if (c == 0) { s->cnt[k]++; return 1; }
        if (c > 0) break;
    }
    if (s->nmsg >= OK_) return 0;
    memmove(&s->msg[k + 1], &s->msg[k], (size_t)(s->nmsg - k) * sizeof(msg_t));
    memmove(&s->cnt[k + 1], &s->cnt[k], (size_t)(s->nmsg - k));
    s->msg[k] = *m;
    s->cnt[k] = 1;
    s->nmsg++;
    return 1;
}

/* WithoutMessage (:92): bag (-) SetToBag({m}); a count reaching 0 removes the key. */
static void bag_remove(ost_t* s, const msg_t* m) {
    for (int k = 0; k < s->nmsg; k++) {
        if (msg_cmp(&s->msg[k], m) == 0) {
            if (--s->cnt[k] == 0) {
                memmove(&s->msg[k], &s->msg[k + 1], (size_t)(s->nmsg - k - 1) * sizeof(msg_t));
                memmove(&s->cnt[k], &s->cnt[k + 1], (size_t)(s->nmsg - k - 1));
                s->nmsg--;
                memset(&s->msg[s->nmsg], 0, sizeof(msg_t));
                s->cnt[s->nmsg] = 0;
            }
            return;
        }
    }
}

static void init_state(const omodel_t* M, ost_t* s) { /* raft.tla:113-129 */
    memset(s, 0, sizeof *s);
    for (int i = 0; i < M->S; i++) {
        s->ct[i] = 1;
        s->st[i] = FOLLOWER;
        s->vf[i] = NIL;
        for (int j = 0; j < M->S; j++) s->ni[i][j] = 1;
    }
}

/* ---------------- successor enumeration (raft.tla:136-430) ---------------- */
typedef struct { ost_t* out; int n; int overflow; } sink_t;

static ost_t* emit(sink_t* k, const ost_t* s) { k->out[k->n] = *s; return &k->out[k->n++]; }

static void send_or_flag(sink_t* k, ost_t* t, const msg_t* m) {
    if (!bag_add(t, m)) k->overflow = 1;
}

/* Receive(m) raft.tla:388-403 for message slot `mk` of s. */
static void receive(const omodel_t* M, const ost_t* s, int mk, sink_t* k) {
    (void)M;
    const msg_t* m = &s->msg[mk];
    int i = m->dst, j = m->src;
    int ct = s->ct[i];
    /* UpdateTerm :373-379 — m is not consumed */
    if (m->term > ct) {
        ost_t* t = emit(k, s);
        t->ct[i] = m->term; t->st[i] = FOLLOWER; t->vf[i] = NIL;
    }
    if (m->type == RVQ && m->term <= ct) { /* HandleRequestVoteRequest :244-263 */
        int lt = last_term(s, i);
        int logok = m->a > lt || (m->a == lt && m->b >= s->len[i]);
        int grant = m->term == ct && logok && (s->vf[i] == NIL || s->vf[i] == j);
        ost_t* t = emit(k, s);
        if (grant) t->vf[i] = (int8_t)j;
        msg_t r; memset(&r, 0, sizeof r);
        r.type = RVP; r.term = (int8_t)ct; r.src = (int8_t)i; r.dst = (int8_t)j;
        r.a = (int8_t)grant; r.n = s->len[i];
        for (int x = 0; x < s->len[i]; x++) r.e[x] = s->log[i][x];
        msg_t req = *m;
        send_or_flag(k, t, &r);     /* Reply :102-103 = add response, then remove request */
        bag_remove(t, &req);
    }
    if (m->type == RVP) {
        if (m->term < ct) { ost_t* t = emit(k, s); msg_t q = *m; bag_remove(t, &q); } /* :382-385 */
        if (m->term == ct) { /* HandleRequestVoteResponse :267-279 */
            ost_t* t = emit(k, s);
            t->vR[i] |= (uint8_t)(1u << j);
            if (m->a) t->vG[i] |= (uint8_t)(1u << j);
            msg_t q = *m; bag_remove(t, &q);
        }
    }
    if (m->type == AEQ && m->term <= ct) { /* HandleAppendEntriesRequest :347-356 */
        int pidx = m->a;
        int logok = pidx == 0 || (pidx > 0 && pidx <= s->len[i] && m->b == s->log[i][pidx - 1].term);
        if (m->term < ct || (m->term == ct && s->st[i] == FOLLOWER && !logok)) { /* Reject :281-293 */
            ost_t* t = emit(k, s);
            msg_t r; memset(&r, 0, sizeof r);
            r.type = AEP; r.term = (int8_t)ct; r.src = (int8_t)i; r.dst = (int8_t)j; r.a = 0; r.b = 0;
            msg_t q = *m;
            send_or_flag(k, t, &r);
            bag_remove(t, &q);
        }
        if (m->term == ct && s->st[i] == CANDIDATE) { /* ReturnToFollowerState :295-299 */
            ost_t* t = emit(k, s);
            t->st[i] = FOLLOWER;
        }
        if (m->term == ct && s->st[i] == FOLLOWER && logok) { /* Accept :333-341 */
            int index = pidx + 1;
            int len = s->len[i];
            /* AppendEntriesAlreadyDone :301-317 (effective guard mcommitIndex = commitIndex[i]) */
            if ((m->n == 0 || (m->n > 0 && len >= index && s->log[i][index - 1].term == m->e[0].term)) &&
                m->c == s->ci[i]) {
                ost_t* t = emit(k, s);
                msg_t r; memset(&r, 0, sizeof r);
                r.type = AEP; r.term = (int8_t)ct; r.src = (int8_t)i; r.dst = (int8_t)j;
                r.a = 1; r.b = (int8_t)(pidx + m->n);
                msg_t q = *m;
                send_or_flag(k, t, &r);
                bag_remove(t, &q);
            }
            /* ConflictAppendEntriesRequest :319-325 — drops the LAST entry, keeps m */
            if (m->n > 0 && len >= index && s->log[i][index - 1].term != m->e[0].term) {
                ost_t* t = emit(k, s);
                t->len[i] = (int8_t)(len - 1);
                t->log[i][len - 1].term = 0; t->log[i][len - 1].value = 0;
            }
            /* NoConflictAppendEntriesRequest :327-331 — keeps m */
            if (m->n > 0 && len == pidx) {
                ost_t* t = emit(k, s);
                if (len >= OL) k->overflow = 1;
                else { t->log[i][len] = m->e[0]; t->len[i] = (int8_t)(len + 1); }
            }
        }
    }
    if (m->type == AEP) {
        if (m->term < ct) { ost_t* t = emit(k, s); msg_t q = *m; bag_remove(t, &q); } /* :382-385 */
        if (m->term == ct) { /* HandleAppendEntriesResponse :360-370 */
            ost_t* t = emit(k, s);
            if (m->a) { t->ni[i][j] = (int8_t)(m->b + 1); t->mi[i][j] = m->b; }
            else { int v = s->ni[i][j] - 1; t->ni[i][j] = (int8_t)(v < 1 ? 1 : v); }
            msg_t q = *m; bag_remove(t, &q);
        }
    }
}

/* All successors of s in the lane-table order of SURVEY.md §2a.  fam[] gets the
 * family id of each successor (0..9 in raft.tla:421-430 order). */
static int successors(const omodel_t* M, const ost_t* s, ost_t* out, int* fam, int* overflow) {
    sink_t k = {out, 0, 0};
    const int S = M->S;
#define MARK(f) do { for (int _q = n0; _q < k.n; _q++) fam[_q] = (f); } while (0)
    int n0;
    n0 = k.n;
    for (int i = 0; i < S; i++) { /* Restart :136-143 */
        ost_t* t = emit(&k, s);
        t->st[i] = FOLLOWER; t->vR[i] = 0; t->vG[i] = 0; t->ci[i] = 0;
        for (int j = 0; j < S; j++) { t->ni[i][j] = 1; t->mi[i][j] = 0; }
    }
    MARK(0); n0 = k.n;
    for (int i = 0; i < S; i++) { /* Timeout :146-154 */
        if (s->st[i] != FOLLOWER && s->st[i] != CANDIDATE) continue;
        ost_t* t = emit(&k, s);
        t->st[i] = CANDIDATE; t->ct[i] = (int8_t)(s->ct[i] + 1); t->vf[i] = NIL; t->vR[i] = 0; t->vG[i] = 0;
    }
    MARK(1); n0 = k.n;
    for (int i = 0; i < S; i++) for (int j = 0; j < S; j++) { /* RequestVote :157-166 */
        if (s->st[i] != CANDIDATE || (s->vR[i] >> j & 1)) continue;
        ost_t* t = emit(&k, s);
        msg_t m; memset(&m, 0, sizeof m);
        m.type = RVQ; m.term = s->ct[i]; m.a = (int8_t)last_term(s, i); m.b = s->len[i];
        m.src = (int8_t)i; m.dst = (int8_t)j;
        send_or_flag(&k, t, &m);
    }
    MARK(2); n0 = k.n;
    for (int i = 0; i < S; i++) { /* BecomeLeader :195-203 */
        if (s->st[i] != CANDIDATE) continue;
        if (M->bug_quorum ? s->vG[i] == 0 : !is_quorum(M, s->vG[i])) continue;
        ost_t* t = emit(&k, s);
        t->st[i] = LEADER;
        for (int j = 0; j < S; j++) { t->ni[i][j] = (int8_t)(s->len[i] + 1); t->mi[i][j] = 0; }
    }
    MARK(3); n0 = k.n;
    for (int i = 0; i < S; i++) for (int v = 0; v < M->V; v++) { /* ClientRequest :206-213 */
        if (s->st[i] != LEADER) continue;
        ost_t* t = emit(&k, s);
        if (s->len[i] >= OL) { k.overflow = 1; continue; }
        t->log[i][s->len[i]].term = s->ct[i]; t->log[i][s->len[i]].value = (int8_t)v;
        t->len[i] = (int8_t)(s->len[i] + 1);
    }
    MARK(4); n0 = k.n;
    for (int i = 0; i < S; i++) { /* AdvanceCommitIndex :219-236 */
        if (s->st[i] != LEADER) continue;
        int best = 0;
        for (int idx = 1; idx <= s->len[i]; idx++) {
            unsigned agree = 1u << i;
            for (int q = 0; q < S; q++) if (s->mi[i][q] >= idx) agree |= 1u << q;
            if (is_quorum(M, agree)) best = idx; /* Max(agreeIndexes) */
        }
        ost_t* t = emit(&k, s);
        if (best > 0 && s->log[i][best - 1].term == s->ct[i]) t->ci[i] = (int8_t)best;
    }
    MARK(5); n0 = k.n;
    for (int i = 0; i < S; i++) for (int j = 0; j < S; j++) { /* AppendEntries :171-192 */
        if (i == j || s->st[i] != LEADER) continue;
        int nidx = s->ni[i][j], len = s->len[i];
        int prev = nidx - 1;
        int prevterm = (prev > 0 && prev <= len) ? s->log[i][prev - 1].term : 0;
        int last = len < nidx ? len : nidx;
        msg_t m; memset(&m, 0, sizeof m);
        m.type = AEQ; m.term = s->ct[i]; m.a = (int8_t)prev; m.b = (int8_t)prevterm;
        if (nidx <= last) { m.n = 1; m.e[0] = s->log[i][nidx - 1]; }
        m.c = (int8_t)(s->ci[i] < last ? s->ci[i] : last);
        m.src = (int8_t)i; m.dst = (int8_t)j;
        ost_t* t = emit(&k, s);
        send_or_flag(&k, t, &m);
    }
    MARK(6); n0 = k.n;
    for (int q = 0; q < s->nmsg; q++) receive(M, s, q, &k); /* Receive :388-403 */
    MARK(7); n0 = k.n;
    for (int q = 0; q < s->nmsg; q++) { ost_t* t = emit(&k, s); t->cnt[q]++; } /* Duplicate :410-412 */
    MARK(8); n0 = k.n;
    for (int q = 0; q < s->nmsg; q++) { ost_t* t = emit(&k, s); msg_t m = s->msg[q]; bag_remove(t, &m); } /* Drop :415-417 */
    MARK(9);
#undef MARK
    *overflow = k.overflow;
    return k.n;
}
#define MAX_SUCC (OS + OS + OS * OS + OS + OS * 4 + OS + OS * OS + 3 * OK_ + 8)

/* ---------------- constraint & invariants ---------------- */
static int in_constraint(const omodel_t* M, const ost_t* s) {
    for (int i = 0; i < M->S; i++) {
        if (M->max_term >= 0 && s->ct[i] > M->max_term) return 0;
        if (M->max_log >= 0 && s->len[i] > M->max_log) return 0;
    }
    if (M->max_msgs >= 0 && s->nmsg > M->max_msgs) return 0;
    if (M->max_dup >= 0)
        for (int q = 0; q < s->nmsg; q++) if (s->cnt[q] > M->max_dup) return 0;
    return 1;
}

static int type_ok(const omodel_t* M, const ost_t* s) { /* raft.tla:482-492 */
    for (int i = 0; i < M->S; i++) {
        if (s->ct[i] < 0 || s->st[i] < 0 || s->st[i] > 2 || s->ci[i] < 0) return 0;
        if (s->vf[i] != NIL && (s->vf[i] < 0 || s->vf[i] >= M->S)) return 0;
        if ((s->vR[i] | s->vG[i]) >> M->S) return 0;
        for (int j = 0; j < M->S; j++) if (s->ni[i][j] < 1 || s->mi[i][j] < 0) return 0;
        for (int x = 0; x < s->len[i]; x++)
            if (s->log[i][x].term < 0 || s->log[i][x].value < 0 || s->log[i][x].value >= M->V) return 0;
    }
    for (int q = 0; q < s->nmsg; q++) {
        const msg_t* m = &s->msg[q];
        if (s->cnt[q] < 1 || m->term < 0 || m->src < 0 || m->src >= M->S || m->dst < 0 || m->dst >= M->S) return 0;
        if (m->type == AEQ && (m->b < 0 || m->c < 0)) return 0;
        if (m->type == RVQ && (m->a < 0 || m->b < 0)) return 0;
        if (m->type == AEP && m->b < 0) return 0;
        for (int x = 0; x < m->n; x++) if (m->e[x].value < 0 || m->e[x].value >= M->V) return 0;
    }
    return 1;
}

static int one_leader_per_term(const omodel_t* M, const ost_t* s) {
    for (int i = 0; i < M->S; i++)
        for (int j = i + 1; j < M->S; j++)
            if (s->st[i] == LEADER && s->st[j] == LEADER && s->ct[i] == s->ct[j]) return 0;
    return 1;
}

static int log_matching(const omodel_t* M, const ost_t* s) { /* raft.tla:1132-1136 */
    for (int i = 0; i < M->S; i++)
        for (int j = 0; j < M->S; j++) {
            int n = s->len[i] < s->len[j] ? s->len[i] : s->len[j];
            for (int x = 1; x <= n; x++)
                if (s->log[i][x - 1].term == s->log[j][x - 1].term &&
                    memcmp(s->log[i], s->log[j], (size_t)x * sizeof(ent_t)) != 0)
                    return 0;
        }
    return 1;
}

/* MessagesInv raft.tla:941-946 over every message of the bag (:910's `m.dest`
 * read as `m.mdest`); log[src][mprevLogIndex + 1] outside DOMAIN log[src] (a TLC
 * evaluation error) counts as a violation. */
static int messages_inv(const omodel_t* M, const ost_t* s) {
    (void)M;
    for (int q = 0; q < s->nmsg; q++) {
        const msg_t* m = &s->msg[q];
        int src = m->src, dst = m->dst, cs = s->ct[src];
        if (m->term > cs) return 0; /* MessageTermsLtCurrentTerm :934-935 */
        if (m->type == RVP && m->a && cs == s->ct[dst] && cs == m->term) { /* :903-910 */
            int ld = last_term(s, dst), ls = last_term(s, src);
            if (!(ld > ls || (ld == ls && s->len[dst] >= s->len[src]))) return 0;
        }
        if (m->type == RVQ && s->st[src] == CANDIDATE && cs == m->term) /* :915-920 */
            if (m->b != s->len[src] || m->a != last_term(s, src)) return 0;
        if (m->type == AEQ && m->n > 0 && m->term == cs) { /* :924-930 */
            int p = m->a; /* mprevLogIndex */
            if (p + 1 < 1 || p + 1 > s->len[src]) return 0;
            if (memcmp(&s->log[src][p], &m->e[0], sizeof(ent_t)) != 0) return 0;
            if (p > 0 && p <= s->len[src] && s->log[src][p - 1].term != m->b) return 0;
        }
    }
    return 1;
}

/* LeaderVotesQuorum raft.tla:1033-1037 */
static int leader_votes_quorum(const omodel_t* M, const ost_t* s) {
    for (int i = 0; i < M->S; i++) {
        if (s->st[i] != LEADER) continue;
        unsigned q = 0;
        for (int j = 0; j < M->S; j++)
            if (s->ct[j] > s->ct[i] || (s->ct[j] == s->ct[i] && s->vf[j] == i)) q |= 1u << j;
        if (!is_quorum(M, q)) return 0;
    }
    return 1;
}

/* CandidateTermNotInLog raft.tla:1041-1047 */
static int candidate_term_not_in_log(const omodel_t* M, const ost_t* s) {
    for (int i = 0; i < M->S; i++) {
        if (s->st[i] != CANDIDATE) continue;
        unsigned q = 0;
        for (int j = 0; j < M->S; j++)
            if (s->ct[j] == s->ct[i] && (s->vf[j] == i || s->vf[j] == NIL)) q |= 1u << j;
        if (!is_quorum(M, q)) continue;
        for (int j = 0; j < M->S; j++)
            for (int n = 0; n < s->len[j]; n++)
                if (s->log[j][n].term == s->ct[i]) return 0;
    }
    return 1;
}

/* The IsPrefix invariants (raft.tla:1143-1180) as restated in
 * specs/MCraftBounded.tla: Committed(j) = the first min(commitIndex[j],
 * Len(log[j])) entries of log[j]; IsPrefix(s, t) = Len(s) <= Len(t) and t
 * starts with s. */
static int committed_prefix_of(const ost_t* s, int j, int i) { /* IsPrefix(Committed(j), log[i]) */
    int c = s->ci[j] < s->len[j] ? s->ci[j] : s->len[j];
    if (s->len[i] < c) return 0;
    return memcmp(s->log[i], s->log[j], (size_t)c * sizeof(ent_t)) == 0;
}
static int votes_granted_inv(const omodel_t* M, const ost_t* s) { /* raft.tla:1145-1153 */
    for (int i = 0; i < M->S; i++)
        for (int j = 0; j < M->S; j++)
            if (((s->vG[i] >> j) & 1u) && s->ct[i] == s->ct[j] && !committed_prefix_of(s, j, i)) return 0;
    return 1;
}
static int quorum_log_inv(const omodel_t* M, const ost_t* s) { /* raft.tla:1157-1161 */
    for (int i = 0; i < M->S; i++) {
        unsigned miss = 0; /* servers whose log lacks Committed(i): no quorum may lie inside */
        for (int j = 0; j < M->S; j++)
            if (!committed_prefix_of(s, i, j)) miss |= 1u << j;
        if (is_quorum(M, miss)) return 0;
    }
    return 1;
}
static int more_up_to_date_correct(const omodel_t* M, const ost_t* s) { /* raft.tla:1167-1172 */
    for (int i = 0; i < M->S; i++)
        for (int j = 0; j < M->S; j++) {
            int li = last_term(s, i), lj = last_term(s, j);
            if ((li > lj || (li == lj && s->len[i] >= s->len[j])) && !committed_prefix_of(s, j, i)) return 0;
        }
    return 1;
}
static int leader_completeness(const omodel_t* M, const ost_t* s) { /* raft.tla:1176-1180 */
    for (int i = 0; i < M->S; i++) {
        if (s->st[i] != LEADER) continue;
        for (int j = 0; j < M->S; j++)
            if (!committed_prefix_of(s, j, i)) return 0;
    }
    return 1;
}

/* returns 0 if ok, else the bit of the first violated invariant */
static int check_invariants(const omodel_t* M, const ost_t* s) {
    if ((M->inv_mask & INV_TYPEOK) && !type_ok(M, s)) return INV_TYPEOK;
    if ((M->inv_mask & INV_ONE_LEADER) && !one_leader_per_term(M, s)) return INV_ONE_LEADER;
    if ((M->inv_mask & INV_LOG_MATCHING) && !log_matching(M, s)) return INV_LOG_MATCHING;
    if ((M->inv_mask & INV_MESSAGES) && !messages_inv(M, s)) return INV_MESSAGES;
    if ((M->inv_mask & INV_LEADER_VOTES) && !leader_votes_quorum(M, s)) return INV_LEADER_VOTES;
    if ((M->inv_mask & INV_CAND_TERM) && !candidate_term_not_in_log(M, s)) return INV_CAND_TERM;
    if ((M->inv_mask & INV_VOTES_GRANTED) && !votes_granted_inv(M, s)) return INV_VOTES_GRANTED;
    if ((M->inv_mask & INV_QUORUM_LOG) && !quorum_log_inv(M, s)) return INV_QUORUM_LOG;
    if ((M->inv_mask & INV_MORE_UP_TO_DATE) && !more_up_to_date_correct(M, s)) return INV_MORE_UP_TO_DATE;
    if ((M->inv_mask & INV_LEADER_COMPLETE) && !leader_completeness(M, s)) return INV_LEADER_COMPLETE;
    return 0;
}

/* ---------------- symmetry: least permuted state (memcmp order) ---------------- */
static void permute(const omodel_t* M, const ost_t* s, const int* p, ost_t* t) {
    int S = M->S, inv[OS];
    for (int a = 0; a < S; a++) inv[p[a]] = a;
    memset(t, 0, sizeof *t);
    for (int i = 0; i < S; i++) {
        int o = inv[i];
        t->ct[i] = s->ct[o]; t->st[i] = s->st[o]; t->ci[i] = s->ci[o]; t->len[i] = s->len[o];
        t->vf[i] = s->vf[o] == NIL ? NIL : (int8_t)p[s->vf[o]];
        memcpy(t->log[i], s->log[o], sizeof(t->log[i]));
        uint8_t r = 0, g = 0;
        for (int q = 0; q < S; q++) {
            if (s->vR[o] >> q & 1) r |= (uint8_t)(1u << p[q]);
            if (s->vG[o] >> q & 1) g |= (uint8_t)(1u << p[q]);
        }
        t->vR[i] = r; t->vG[i] = g;
        for (int j = 0; j < S; j++) { t->ni[i][j] = s->ni[o][inv[j]]; t->mi[i][j] = s->mi[o][inv[j]]; }
    }
    for (int q = 0; q < s->nmsg; q++) {
        msg_t m = s->msg[q];
        m.src = (int8_t)p[m.src]; m.dst = (int8_t)p[m.dst];
        int k;
        for (k = 0; k < t->nmsg; k++) if (msg_cmp(&t->msg[k], &m) > 0) break;
        memmove(&t->msg[k + 1], &t->msg[k], (size_t)(t->nmsg - k) * sizeof(msg_t));
        memmove(&t->cnt[k + 1], &t->cnt[k], (size_t)(t->nmsg - k));
        t->msg[k] = m; t->cnt[k] = s->cnt[q]; t->nmsg++;
    }
}

static int n_perms;
static int perms[120][OS];
static void gen_perms(int S) {
    int a[OS] = {0};
    for (int i = 0; i < S; i++) a[i] = i;
    n_perms = 0;
    for (;;) {
        memcpy(perms[n_perms++], a, sizeof a);
        int i = S - 2;
        while (i >= 0 && a[i] > a[i + 1]) i--;
        if (i < 0) break;
        int j = S - 1;
        while (a[j] < a[i]) j--;
        int x = a[i]; a[i] = a[j]; a[j] = x;
        for (int l = i + 1, r = S - 1; l < r; l++, r--) { x = a[l]; a[l] = a[r]; a[r] = x; }
    }
}

static void canonicalize(const omodel_t* M, const ost_t* s, ost_t* out) {
    ost_t t;
    *out = *s;
    for (int q = 1; q < n_perms; q++) {
        permute(M, s, perms[q], &t);
        if (memcmp(&t, out, sizeof t) < 0) *out = t;
    }
}

/* ---------------- exact concurrent state set ---------------- */
static uint64_t hash_bytes(const void* p, size_t n) {
    const unsigned char* c = (const unsigned char*)p;
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (size_t k = 0; k + 8 <= n; k += 8) {
        uint64_t x;
        memcpy(&x, c + k, 8);
        x *= 0xbf58476d1ce4e5b9ull;
        x ^= x >> 31;
        h = (h ^ x) * 0x94d049bb133111ebull;
        h ^= h >> 29;
    }
    return h;
}

#define NSHARD 4096
typedef struct {
    pthread_mutex_t mu;
    uint64_t* slot; /* state index + 1, 0 = empty */
    uint64_t cap, used;
} shard_t;

typedef struct {
    omodel_t M;
    ost_t* states;     /* all distinct states (the stored, non-canonical member) */
    ost_t* keys;       /* canonical keys when symmetry is on (else == states) */
    uint64_t* parent;
    uint64_t cap, count;
    shard_t sh[NSHARD];
} oset_t;

static int oset_insert(oset_t* O, const ost_t* key, const ost_t* st, uint64_t parent, uint64_t* idx_out) {
    uint64_t h = hash_bytes(key, sizeof *key);
    shard_t* S = &O->sh[h & (NSHARD - 1)];
    pthread_mutex_lock(&S->mu);
    if ((S->used + 1) * 2 > S->cap) { /* grow */
        uint64_t ncap = S->cap ? S->cap * 2 : 64;
        uint64_t* ns = calloc(ncap, sizeof(uint64_t));
        for (uint64_t q = 0; q < S->cap; q++) {
            uint64_t v = S->slot[q];
            if (!v) continue;
            uint64_t hh = hash_bytes(&O->keys[v - 1], sizeof(ost_t)) >> 12;
            uint64_t p = hh & (ncap - 1);
            while (ns[p]) p = (p + 1) & (ncap - 1);
            ns[p] = v;
        }
        free(S->slot);
        S->slot = ns; S->cap = ncap;
    }
    uint64_t p = (h >> 12) & (S->cap - 1);
    for (;;) {
        uint64_t v = S->slot[p];
        if (!v) break;
        if (memcmp(&O->keys[v - 1], key, sizeof *key) == 0) { pthread_mutex_unlock(&S->mu); return 0; }
        p = (p + 1) & (S->cap - 1);
    }
    uint64_t idx = __atomic_fetch_add(&O->count, 1, __ATOMIC_RELAXED);
    if (idx >= O->cap) { pthread_mutex_unlock(&S->mu); return -1; }
    O->states[idx] = *st;
    if (O->keys != O->states) O->keys[idx] = *key;
    O->parent[idx] = parent;
    S->slot[p] = idx + 1;
    S->used++;
    pthread_mutex_unlock(&S->mu);
    *idx_out = idx;
    return 1;
}

/* ---------------- BFS driver ---------------- */
typedef struct {
    uint64_t generated, distinct, left_on_queue;
    int32_t depth, violated_inv, violation_depth, overflow;
    uint64_t violation_index;
    double seconds;
} orc_result;

typedef struct {
    oset_t* O;
    uint64_t lo, hi;
    uint64_t next; /* work-stealing cursor */
    uint64_t gen;
    int viol;
    uint64_t viol_idx;
    int overflow;
    pthread_mutex_t mu;
} level_t;

static void* worker(void* arg) {
    level_t* L = (level_t*)arg;
    oset_t* O = L->O;
    ost_t* out = malloc(sizeof(ost_t) * MAX_SUCC);
    int fam[MAX_SUCC];
    uint64_t gen = 0;
    int overflow = 0, viol = 0;
    uint64_t viol_idx = 0;
    for (;;) {
        uint64_t b = __atomic_fetch_add(&L->next, 256, __ATOMIC_RELAXED);
        if (b >= L->hi) break;
        uint64_t e = b + 256 < L->hi ? b + 256 : L->hi;
        for (uint64_t x = b; x < e; x++) {
            int ov = 0;
            int n = successors(&O->M, &O->states[x], out, fam, &ov);
            gen += (uint64_t)n;
            for (int q = 0; q < n; q++) {
                if (!in_constraint(&O->M, &out[q])) continue;
                ost_t key;
                const ost_t* kp = &out[q];
                if (O->M.symmetry) { canonicalize(&O->M, &out[q], &key); kp = &key; }
                uint64_t idx;
                int r = oset_insert(O, kp, &out[q], x, &idx);
                if (r < 0) { overflow = 1; continue; }
                if (r == 1) {
                    int v = check_invariants(&O->M, &out[q]);
                    if (v && (!viol || idx < viol_idx)) { viol = v; viol_idx = idx; }
                }
            }
            if (ov) overflow = 1;
        }
    }
    pthread_mutex_lock(&L->mu);
    L->gen += gen;
    if (overflow) L->overflow = 1;
    if (viol && (!L->viol || viol_idx < L->viol_idx)) { L->viol = viol; L->viol_idx = viol_idx; }
    pthread_mutex_unlock(&L->mu);
    free(out);
    return NULL;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* Exported for ctypes.  level_new/level_gen (may be NULL) receive per-level
 * counts (index d-1 = level d; level_gen[d] = successors generated by
 * expanding level d, level_gen[0] = initial states), up to max_out entries.
 * A negative bound means "unbounded".  Returns 0 on success. */
int orc_bfs(int S, int V, int max_term, int max_log, int max_msgs, int max_dup, int bug_quorum,
            int inv_mask, int symmetry, int threads, int max_levels, uint64_t capacity,
            orc_result* res, uint64_t* level_new, uint64_t* level_gen, int max_out) {
    if (S < 1 || S > OS || V < 1 || V > 4 || threads < 1) return -22;
    if (max_log >= OL || max_msgs >= OK_) return -22;
    oset_t* O = calloc(1, sizeof(oset_t));
    if (!O) return -12;
    omodel_t M = {S, V, max_term, max_log, max_msgs, max_dup, bug_quorum, inv_mask, symmetry};
    O->M = M;
    gen_perms(S);
    O->cap = capacity ? capacity : (1u << 22);
    O->states = malloc(sizeof(ost_t) * O->cap);
    O->keys = symmetry ? malloc(sizeof(ost_t) * O->cap) : O->states;
    O->parent = malloc(sizeof(uint64_t) * O->cap);
    if (!O->states || !O->keys || !O->parent) return -12;
    for (int q = 0; q < NSHARD; q++) pthread_mutex_init(&O->sh[q].mu, NULL);
    memset(res, 0, sizeof *res);
    double t0 = now_s();

    ost_t init, key;
    init_state(&M, &init);
    const ost_t* kp = &init;
    if (symmetry) { canonicalize(&M, &init, &key); kp = &key; }
    uint64_t idx;
    oset_insert(O, kp, &init, UINT64_MAX, &idx);
    res->generated = 1;
    int v0 = check_invariants(&M, &init);
    uint64_t lo = 0, hi = O->count;
    int depth = 1;
    if (level_new && max_out > 0) level_new[0] = 1;
    if (level_gen && max_out > 0) level_gen[0] = 1;
    if (v0) { res->violated_inv = v0; res->violation_depth = 1; res->violation_index = 0; }
    while (!v0 && lo < hi && (max_levels <= 0 || depth < max_levels)) {
        level_t L;
        memset(&L, 0, sizeof L);
        L.O = O; L.lo = lo; L.hi = hi; L.next = lo;
        pthread_mutex_init(&L.mu, NULL);
        pthread_t th[256];
        int nt = threads > 256 ? 256 : threads;
        for (int q = 0; q < nt; q++) pthread_create(&th[q], NULL, worker, &L);
        for (int q = 0; q < nt; q++) pthread_join(th[q], NULL);
        res->generated += L.gen;
        if (level_gen && depth < max_out) level_gen[depth] = L.gen;
        if (L.overflow) { res->overflow = 1; break; }
        uint64_t nhi = O->count;
        if (nhi > hi) {
            depth++;
            if (level_new && depth - 1 < max_out) level_new[depth - 1] = nhi - hi;
        }
        lo = hi; hi = nhi;
        if (L.viol) {
            res->violated_inv = L.viol; res->violation_depth = depth; res->violation_index = L.viol_idx;
            break;
        }
    }
    res->distinct = O->count;
    res->depth = depth;
    res->left_on_queue = hi - lo;
    res->seconds = now_s() - t0;
    for (int q = 0; q < NSHARD; q++) free(O->sh[q].slot);
    if (O->keys != O->states) free(O->keys);
    free(O->states); free(O->parent); free(O);
    return 0;
}

#ifndef ORC_NO_MAIN
int main(int argc, char** argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s S V MaxTerm MaxLog MaxMsgs MaxDup [threads] [max_levels] "
                        "[bug_quorum] [inv_mask] [symmetry] [capacity]\n", argv[0]);
        return 2;
    }
    int S = atoi(argv[1]), V = atoi(argv[2]);
    int mt = atoi(argv[3]), ml = atoi(argv[4]), mm = atoi(argv[5]), md = atoi(argv[6]);
    int th = argc > 7 ? atoi(argv[7]) : 1;
    int lv = argc > 8 ? atoi(argv[8]) : 0;
    int bug = argc > 9 ? atoi(argv[9]) : 0;
    int inv = argc > 10 ? atoi(argv[10]) : INV_TYPEOK;
    int sym = argc > 11 ? atoi(argv[11]) : 0;
    uint64_t cap = argc > 12 ? strtoull(argv[12], NULL, 10) : (1ull << 24);
    orc_result r;
    static uint64_t ln[512], lg[512];
    int rc = orc_bfs(S, V, mt, ml, mm, md, bug, inv, sym, th, lv, cap, &r, ln, lg, 512);
    if (rc) { fprintf(stderr, "error %d\n", rc); return 1; }
    for (int d = 0; d < r.depth && d < 512; d++)
        printf("level %d: new %llu, generated-by-expanding %llu\n", d + 1,
               (unsigned long long)ln[d], (unsigned long long)lg[d + 1 < 512 ? d + 1 : d]);
    printf("%llu states generated, %llu distinct states found, %llu states left on queue.\n",
           (unsigned long long)r.generated, (unsigned long long)r.distinct,
           (unsigned long long)r.left_on_queue);
    printf("The depth of the complete state graph search is %d.\n", r.depth);
    if (r.violated_inv) printf("Invariant violated (mask %d) at depth %d\n", r.violated_inv, r.violation_depth);
    if (r.overflow) printf("OVERFLOW (capacity)\n");
    printf("seconds %.3f  distinct/s %.0f  threads %d\n", r.seconds, r.distinct / r.seconds, th);
    return 0;
}
#endif
