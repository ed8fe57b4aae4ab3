/*
 * ref_cpu.c -- CPU restatement of the reference linearisability search.
 *
 * TEST INFRASTRUCTURE ONLY (the checker and the CPU baseline, "kind: port").
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product path never calls it.
 *
 * Restates src/Linearisability.hs:25-69 of advancedtelematic/
 * quickcheck-state-machine-distributed over the counter state of SURVEY.md
 * §8a Lemma L1 instead of rebuilt cons lists:
 *
 *   - filter1 (:41,:47-50) always drops the FIRST remaining invocation of the
 *     candidate's pid and findResponse (:30-34) the FIRST remaining response
 *     of that pid, so the remaining history is a function of the per-pid
 *     counter vector k: pid p has lost exactly its first k[p] invocations and
 *     first k[p] responses.
 *   - takeInvocations (:25-28): candidates are the remaining invocations
 *     before the first remaining response R = min_p resp_pos[p][k[p]], in
 *     ascending history position; the child of candidate e (pid p) is
 *     Operation p inv_e resp_p[k[p]] (Q1: the node carries the candidate's own
 *     inv even when the removed invocation is an earlier one of the same pid),
 *     and it exists only if p still has a response.
 *   - linearisable (:59-61): [] => True; else plain `any` over the roots
 *     (no roots => False); step (:63-65) = postcondition && any' over the
 *     children where any' [] = True (:67-69).  One node = one step call.
 *
 * Models: test/Bank.hs:92-131 (next', invariant, post; Map.! raises ->
 * model error) and test/TicketDispenser.hs:81-102.  Encoding: include/qsmd.h.
 */
#include "qsmd.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint32_t exists;
    int64_t bal[QSMD_BANK_MAX_ACCOUNTS];
} bank_m;

typedef struct {
    int is_just;
    int64_t n;
} ticket_m;

typedef union {
    bank_m bank;
    ticket_m ticket;
} model_u;

enum { R_FALSE = 0, R_TRUE = 1, R_ERROR = 2, R_BUDGET = 3 };

typedef struct {
    uint32_t model_id;
    const qsmd_event* ev;
    int n_ev;
    int n_pid;
    /* per event */
    uint8_t pid[QSMD_MAX_EVENTS];
    uint8_t is_resp[QSMD_MAX_EVENTS];
    uint8_t ord[QSMD_MAX_EVENTS];        /* ordinal among (pid, kind) */
    /* per pid */
    uint8_t nresp[QSMD_MAX_PIDS];
    uint8_t resp_start[QSMD_MAX_PIDS];
    uint8_t resp_pos[QSMD_MAX_EVENTS];   /* flattened per-pid lists */
    uint8_t k[QSMD_MAX_PIDS];
    /* search */
    uint64_t nodes, max_nodes;
    uint8_t path[QSMD_MAX_EVENTS];
    int depth;
    struct memo_t* memo;                 /* QSMD_FLAG_MEMO: failed states, or NULL */
} search_t;

/* ------------------------------------------------------------- memo */
/* QSMD_FLAG_MEMO restated: a state (counter vector k, model) whose subtree
 * was searched completely without success is remembered; reaching it again
 * counts the node (its postcondition was evaluated) and skips the subtree.
 * The outcome of a subtree is a function of the state alone (Lemma L1), so
 * verdicts are those of the exhaustive search. */
#define MEMO_KEY (QSMD_MAX_PIDS + 1 + 8 * 9)
typedef struct memo_t {
    uint8_t* keys;     /* cap x MEMO_KEY */
    uint8_t* used;
    uint64_t cap, n;
} memo_t;

static uint64_t memo_hash(const uint8_t* k) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < MEMO_KEY; ++i) { h ^= k[i]; h *= 1099511628211ull; }
    return h;
}

static void memo_key(const search_t* s, const model_u* m, uint8_t* k) {
    memset(k, 0, MEMO_KEY);
    memcpy(k, s->k, (size_t)s->n_pid);
    uint8_t* q = k + QSMD_MAX_PIDS;
    if (s->model_id == QSMD_MODEL_BANK) {
        q[0] = (uint8_t)m->bank.exists;
        for (int a = 0; a < QSMD_BANK_MAX_ACCOUNTS; ++a) memcpy(q + 1 + 8 * a, &m->bank.bal[a], 8);
    } else {
        q[0] = (uint8_t)m->ticket.is_just;
        memcpy(q + 1, &m->ticket.n, 8);
    }
}

static int memo_find(memo_t* t, const uint8_t* k, int insert) {
    if (insert && 2 * (t->n + 1) > t->cap) {             /* grow: rehash */
        memo_t u = {0};
        u.cap = t->cap ? 2 * t->cap : 1024;
        u.keys = (uint8_t*)malloc(u.cap * MEMO_KEY);
        u.used = (uint8_t*)calloc(u.cap, 1);
        for (uint64_t i = 0; i < t->cap; ++i)
            if (t->used[i]) memo_find(&u, t->keys + i * MEMO_KEY, 1);
        free(t->keys);
        free(t->used);
        *t = u;
    }
    if (!t->cap) return 0;
    for (uint64_t i = memo_hash(k) & (t->cap - 1);; i = (i + 1) & (t->cap - 1)) {
        if (!t->used[i]) {
            if (!insert) return 0;
            memcpy(t->keys + i * MEMO_KEY, k, MEMO_KEY);
            t->used[i] = 1;
            t->n++;
            return 1;
        }
        if (memcmp(t->keys + i * MEMO_KEY, k, MEMO_KEY) == 0) return 1;
    }
}

/* ------------------------------------------------------------- models */

/* test/Bank.hs:103-104 */
static int bank_invariant(const bank_m* m) {
    for (int a = 0; a < QSMD_BANK_MAX_ACCOUNTS; ++a)
        if (((m->exists >> a) & 1u) && m->bal[a] < 0) return 0;
    return 1;
}

/* M.lookup acc model >= Just money   (Nothing < Just _) */
static int bank_ge(const bank_m* m, int a, int64_t money) {
    return ((m->exists >> a) & 1u) && m->bal[a] >= money;
}

/* test/Bank.hs:118-131.  Returns R_FALSE / R_TRUE / R_ERROR. */
static int bank_post(const bank_m* m, const qsmd_event* inv, const qsmd_event* resp) {
    if (!bank_invariant(m)) return R_FALSE;
    int a = inv->a;
    switch (inv->code) {
    case QSMD_BANK_OPEN_ACCOUNT:
        return resp->code == (((m->exists >> a) & 1u) ? QSMD_BANK_ACCOUNT_ALREADY_EXISTS
                                                       : QSMD_BANK_ACCOUNT_CREATED);
    case QSMD_BANK_DEPOSIT:
        return resp->code == QSMD_BANK_DEPOSIT_MADE;
    case QSMD_BANK_WITHDRAW:
        return resp->code == (bank_ge(m, a, inv->val) ? QSMD_BANK_WITHDRAWAL_MADE
                                                      : QSMD_BANK_INSUFFICIENT_FUNDS);
    case QSMD_BANK_CHECK_BALANCE:
        /* resp == Balance (model M.! acc): derived Eq forces the field only
         * when resp is a Balance (test/Bank.hs:128). */
        if (resp->code != QSMD_BANK_BALANCE) return R_FALSE;
        if (!((m->exists >> a) & 1u)) return R_ERROR;
        return (int64_t)resp->val == m->bal[a];
    case QSMD_BANK_TRANSFER:
        return resp->code == (bank_ge(m, a, inv->val) ? QSMD_BANK_TRANSFER_MADE
                                                      : QSMD_BANK_INSUFFICIENT_FUNDS);
    }
    return R_FALSE;
}

static void bank_deposit(bank_m* m, int a, int64_t money) {   /* insertWith (+) */
    m->bal[a] = ((m->exists >> a) & 1u) ? m->bal[a] + money : money;
    m->exists |= 1u << a;
}
static void bank_withdraw(bank_m* m, int a, int64_t money) {  /* insertWith (\n o -> o - n) */
    m->bal[a] = ((m->exists >> a) & 1u) ? m->bal[a] - money : money;
    m->exists |= 1u << a;
}

/* test/Bank.hs:92-101, applied to a Left request (Right is the identity). */
static void bank_next(bank_m* m, const qsmd_event* inv) {
    int a = inv->a;
    switch (inv->code) {
    case QSMD_BANK_OPEN_ACCOUNT:
        if (!((m->exists >> a) & 1u)) { m->exists |= 1u << a; m->bal[a] = 0; }
        break;
    case QSMD_BANK_DEPOSIT:  bank_deposit(m, a, inv->val); break;
    case QSMD_BANK_WITHDRAW: bank_withdraw(m, a, inv->val); break;
    case QSMD_BANK_CHECK_BALANCE: break;
    case QSMD_BANK_TRANSFER:
        bank_withdraw(m, a, inv->val);
        bank_deposit(m, inv->b, inv->val);
        break;
    }
}

/* test/TicketDispenser.hs:99-102 */
static int ticket_post(const ticket_m* m, const qsmd_event* inv, const qsmd_event* resp) {
    if (inv->code == QSMD_TICKET_TAKE_TICKET && resp->code == QSMD_TICKET_NUMBER)
        return m->is_just && (int64_t)resp->val == m->n + 1;
    if (inv->code == QSMD_TICKET_RESET && resp->code == QSMD_TICKET_OK)
        return R_TRUE;
    return R_FALSE;
}

/* test/TicketDispenser.hs:81-85 */
static void ticket_next(ticket_m* m, const qsmd_event* inv) {
    if (inv->code == QSMD_TICKET_TAKE_TICKET) {
        if (m->is_just) m->n += 1;
    } else {
        m->is_just = 1;
        m->n = 0;
    }
}

/* --------------------------------------------------------- validation */

/* Returns 1 if the history is well-encoded for model_id (include/qsmd.h). */
static int valid_history(uint32_t model_id, const qsmd_hdr* h, const qsmd_event* ev) {
    if (h->model_id != model_id) return 0;
    if (h->n_ev > QSMD_MAX_EVENTS) return 0;
    if (h->n_pid > QSMD_MAX_PIDS) return 0;
    for (int e = 0; e < h->n_ev; ++e) {
        const qsmd_event* x = &ev[e];
        int pid = x->kp & QSMD_EV_PID_MASK;
        int resp = (x->kp & QSMD_EV_RESP) != 0;
        if (pid >= h->n_pid) return 0;
        if (model_id == QSMD_MODEL_TICKET) {
            if (x->code > 1) return 0;
        } else if (model_id == QSMD_MODEL_BANK) {
            if (resp) {
                if (x->code > QSMD_BANK_BALANCE) return 0;
            } else {
                if (x->code > QSMD_BANK_TRANSFER) return 0;
                if (x->a >= QSMD_BANK_MAX_ACCOUNTS) return 0;
                if (x->code == QSMD_BANK_TRANSFER && x->b >= QSMD_BANK_MAX_ACCOUNTS) return 0;
            }
        } else {
            return 0;
        }
    }
    return 1;
}

/* ------------------------------------------------------------- search */

static int post_of(search_t* s, const model_u* m, const qsmd_event* inv, const qsmd_event* resp) {
    if (s->model_id == QSMD_MODEL_BANK) return bank_post(&m->bank, inv, resp);
    return ticket_post(&m->ticket, inv, resp);
}

static void next_of(search_t* s, model_u* m, const qsmd_event* inv) {
    /* transition (transition model (Left inv)) (Right resp): Right is id. */
    if (s->model_id == QSMD_MODEL_BANK) bank_next(&m->bank, inv);
    else ticket_next(&m->ticket, inv);
}

static int expand(search_t* s, const model_u* m, int is_root);

/* step (src/Linearisability.hs:63-65) for the node Operation p inv_e resp_r. */
static int step(search_t* s, const model_u* m, int p, int e, int r) {
    if (s->max_nodes && s->nodes >= s->max_nodes) return R_BUDGET;
    s->nodes++;
    int ok = post_of(s, m, &s->ev[e], &s->ev[r]);
    if (ok != R_TRUE) return ok;           /* False or model error */
    model_u m2 = *m;
    next_of(s, &m2, &s->ev[e]);
    s->path[s->depth++] = (uint8_t)e;
    s->k[p]++;
    int res;
    uint8_t key[MEMO_KEY];
    if (s->memo) memo_key(s, &m2, key);
    if (s->memo && memo_find(s->memo, key, 0)) {
        res = R_FALSE;                               /* known to fail */
    } else {
        res = expand(s, &m2, 0);
        if (s->memo && res == R_FALSE) memo_find(s->memo, key, 1);
    }
    s->k[p]--;
    if (res != R_TRUE) s->depth--;
    return res;
}

/* interleavings at counter state s->k, folded with `any` (root) or `any'`. */
static int expand(search_t* s, const model_u* m, int is_root) {
    int R = s->n_ev;
    for (int p = 0; p < s->n_pid; ++p)
        if (s->k[p] < s->nresp[p]) {
            int pos = s->resp_pos[s->resp_start[p] + s->k[p]];
            if (pos < R) R = pos;
        }
    int any_child = 0;
    for (int e = 0; e < R; ++e) {
        if (s->is_resp[e]) continue;                 /* cannot happen before R */
        int p = s->pid[e];
        if (s->ord[e] < s->k[p]) continue;           /* already removed       */
        if (s->k[p] >= s->nresp[p]) continue;        /* findResponse => []    */
        any_child = 1;
        int r = s->resp_pos[s->resp_start[p] + s->k[p]];
        int res = step(s, m, p, e, r);
        if (res != R_FALSE) return res;              /* True, error, budget   */
    }
    if (!any_child) return is_root ? R_FALSE : R_TRUE;
    return R_FALSE;
}

static void model_init(uint32_t model_id, const void* model0, model_u* m) {
    memset(m, 0, sizeof(*m));
    if (!model0) return;
    if (model_id == QSMD_MODEL_BANK) {
        const qsmd_bank_model* b = (const qsmd_bank_model*)model0;
        m->bank.exists = b->exists;
        for (int a = 0; a < QSMD_BANK_MAX_ACCOUNTS; ++a)
            m->bank.bal[a] = ((b->exists >> a) & 1u) ? b->balance[a] : 0;
    } else {
        const qsmd_ticket_model* t = (const qsmd_ticket_model*)model0;
        m->ticket.is_just = t->is_just ? 1 : 0;
        m->ticket.n = t->is_just ? t->n : 0;
    }
}

/* Check one history.  Returns the QSMD_STATUS_* code. */
static uint8_t check_one(uint32_t model_id, const qsmd_hdr* h, const qsmd_event* events,
                         const void* model0, uint64_t max_nodes, uint64_t* nodes_out,
                         uint8_t* witness, memo_t* memo);

uint8_t oracle_check_one(uint32_t model_id, const qsmd_hdr* h, const qsmd_event* events,
                         const void* model0, uint64_t max_nodes,
                         uint64_t* nodes_out, uint8_t* witness /* n_ev bytes or NULL */) {
    return check_one(model_id, h, events, model0, max_nodes, nodes_out, witness, NULL);
}

static uint8_t check_one(uint32_t model_id, const qsmd_hdr* h, const qsmd_event* events,
                         const void* model0, uint64_t max_nodes, uint64_t* nodes_out,
                         uint8_t* witness, memo_t* memo) {
    const qsmd_event* ev = events + h->ev_off;
    *nodes_out = 0;
    if (!valid_history(model_id, h, ev)) return QSMD_STATUS_ENCODE_ERROR;
    if (h->n_ev == 0) {
        return QSMD_STATUS_LINEARISABLE;             /* :59 */
    }
    search_t s;
    s.model_id = model_id;
    s.ev = ev;
    s.n_ev = h->n_ev;
    s.n_pid = h->n_pid;
    s.nodes = 0;
    s.max_nodes = max_nodes;
    s.depth = 0;
    s.memo = memo;
    uint8_t ninv[QSMD_MAX_PIDS];
    memset(ninv, 0, sizeof(ninv));
    memset(s.nresp, 0, sizeof(s.nresp));
    memset(s.k, 0, sizeof(s.k));
    for (int e = 0; e < s.n_ev; ++e) {
        int p = ev[e].kp & QSMD_EV_PID_MASK;
        int rsp = (ev[e].kp & QSMD_EV_RESP) != 0;
        s.pid[e] = (uint8_t)p;
        s.is_resp[e] = (uint8_t)rsp;
        s.ord[e] = rsp ? s.nresp[p]++ : ninv[p]++;
    }
    int off = 0;
    for (int p = 0; p < s.n_pid; ++p) { s.resp_start[p] = (uint8_t)off; off += s.nresp[p]; }
    uint8_t fill[QSMD_MAX_PIDS];
    memset(fill, 0, sizeof(fill));
    for (int e = 0; e < s.n_ev; ++e)
        if (s.is_resp[e]) { int p = s.pid[e]; s.resp_pos[s.resp_start[p] + fill[p]++] = (uint8_t)e; }

    model_u m;
    model_init(model_id, model0, &m);
    int res = expand(&s, &m, 1);
    *nodes_out = s.nodes;
    switch (res) {
    case R_TRUE:
        if (witness) {
            for (int d = 0; d < s.depth; ++d) witness[d] = s.path[d];
            if (s.depth < s.n_ev) witness[s.depth] = QSMD_WITNESS_END;
        }
        return QSMD_STATUS_LINEARISABLE;
    case R_ERROR: return QSMD_STATUS_MODEL_ERROR;
    case R_BUDGET: return QSMD_STATUS_BUDGET;
    default: return QSMD_STATUS_NONLINEARISABLE;
    }
}

/* ---------------------------------------------------------------- batch */

typedef struct {
    uint32_t model_id;
    const qsmd_hdr* hdr;
    const qsmd_event* events;
    const void* model0;
    uint64_t max_nodes;
    uint8_t* status;
    uint64_t* nodes;
    uint8_t* witness;
    uint64_t lo, hi;
    int memo;
} job_t;

static void* run_job(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        uint64_t n = 0;
        uint8_t* w = j->witness ? j->witness + j->hdr[i].ev_off : NULL;
        memo_t m = {0};
        j->status[i] = check_one(j->model_id, &j->hdr[i], j->events, j->model0,
                                 j->max_nodes, &n, w, j->memo ? &m : NULL);
        free(m.keys);
        free(m.used);
        if (j->nodes) j->nodes[i] = n;
    }
    return NULL;
}

/* Check histories [0, n_hist) with n_threads host threads (history shards).
 * Witness (nullable) is indexed like the events array. Returns 0. */
int oracle_check_batch_flags(uint32_t model_id, const qsmd_hdr* hdr, uint64_t n_hist,
                             const qsmd_event* events, const void* model0, uint64_t max_nodes,
                             uint8_t* status, uint64_t* nodes, uint8_t* witness, int n_threads,
                             uint32_t flags);

int oracle_check_batch(uint32_t model_id, const qsmd_hdr* hdr, uint64_t n_hist,
                       const qsmd_event* events, const void* model0, uint64_t max_nodes,
                       uint8_t* status, uint64_t* nodes, uint8_t* witness, int n_threads) {
    return oracle_check_batch_flags(model_id, hdr, n_hist, events, model0, max_nodes, status, nodes,
                                    witness, n_threads, 0);
}

/* flags: QSMD_FLAG_MEMO prunes known-failing states (verdicts only). */
int oracle_check_batch_flags(uint32_t model_id, const qsmd_hdr* hdr, uint64_t n_hist,
                             const qsmd_event* events, const void* model0, uint64_t max_nodes,
                             uint8_t* status, uint64_t* nodes, uint8_t* witness, int n_threads,
                             uint32_t flags) {
    if (n_threads < 1) n_threads = 1;
    if ((uint64_t)n_threads > n_hist) n_threads = n_hist ? (int)n_hist : 1;
    job_t jobs[256];
    pthread_t th[256];
    if (n_threads > 256) n_threads = 256;
    uint64_t per = (n_hist + n_threads - 1) / n_threads;
    for (int t = 0; t < n_threads; ++t) {
        jobs[t] = (job_t){model_id, hdr, events, model0, max_nodes, status, nodes, witness,
                          t * per, (t + 1) * per > n_hist ? n_hist : (t + 1) * per,
                          (flags & QSMD_FLAG_MEMO) != 0};
        if (jobs[t].lo > jobs[t].hi) jobs[t].lo = jobs[t].hi;
    }
    if (n_threads == 1) { run_job(&jobs[0]); return 0; }
    for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, run_job, &jobs[t]);
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    return 0;
}
