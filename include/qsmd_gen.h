/*
 * qsmd_gen.h -- seeded synthetic history generator (C ABI).
 *
 * Produces batches in the include/qsmd.h layout.  It restates the delivery
 * policy of the reference's deterministic scheduler (src/Scheduler.hs:105-186:
 * one mailbox per (client, server) pair, requests and responses of a pair
 * strictly alternate, every tick delivers one event of a uniformly chosen
 * ready pair), the sequential prefix of prop_bank / prop_ticketDispenserParallel
 * (SchedulerSequential, test/Bank.hs:267-269, test/TicketDispenser.hs:294-297)
 * and the request distributions of test/Bank.hs:133-146 (Open:Deposit:
 * Withdraw:Transfer:CheckBalance = 1:5:5:8:5, money getPositive ~ U{1..100})
 * and test/TicketDispenser.hs:108-112 (Reset:TakeTicket = 1:8).
 *
 * Responses come from a sequentially executed implementation of the model
 * (the spec), applied at each operation's linearisation point; so histories
 * are linearisable unless a bug is injected (p_bug).  Each history's RNG is
 * derived from (seed, global history index) only, so any shard of a batch can
 * be generated independently and reproducibly on any rank.
 */
#ifndef QSMD_GEN_H
#define QSMD_GEN_H

#include "qsmd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Linearisation point of the implementation. */
#define QSMD_GEN_LIN_AT_INVOKE 0u  /* actor executes on delivery of the request
                                      (bankSM / clientSM, test/Bank.hs:217-242) */
#define QSMD_GEN_LIN_IN_WINDOW 1u  /* uniformly inside [invoke, response)       */

#define QSMD_GEN_PID_PER_CLIENT 0u /* Bank: pid = account (fromPid, Bank.hs:54)  */
#define QSMD_GEN_PID_SHARED     1u /* TicketDispenser: every event carries the
                                      test process's pid (Q1, TicketDispenser.hs:302-309) */

typedef struct qsmd_gen_params {
    uint32_t model_id;     /* QSMD_MODEL_BANK / QSMD_MODEL_TICKET                 */
    uint32_t n_clients;    /* C: Bank accounts / Ticket clients (<= 8)            */
    uint32_t n_ops;        /* K: total operations per history (<= 64)             */
    uint32_t prefix_ops;   /* sequential prefix (Bank: >= C, opens the accounts)  */
    uint32_t lin_policy;   /* QSMD_GEN_LIN_*                                       */
    uint32_t pid_mode;     /* QSMD_GEN_PID_*                                       */
    uint32_t overlap;      /* max operations outstanding at once (0 = C)          */
    uint32_t money_max;    /* Bank money ~ U{1..money_max} (0 = 100)              */
    double   p_bug;        /* probability of one injected response bug           */
    uint64_t seed;
} qsmd_gen_params;

/* Generate histories [first, first + n_hist) of the stream defined by p.
 * Every history has exactly 2*n_ops events; hdr[i].ev_off = (i * 2 * n_ops)
 * + ev_base.  events must hold n_hist * 2 * n_ops entries.  bug_out
 * (nullable) receives 1 for histories that carry an injected bug.
 * Returns 0, or QSMD_ERR_ARG. */
int qsmd_gen_batch(const qsmd_gen_params* p, uint64_t first, uint64_t n_hist,
                   uint32_t ev_base, qsmd_hdr* hdr, qsmd_event* events,
                   uint8_t* bug_out, int n_threads);

/* On-device generation (libqsmd.so, csrc/gen.hip): the same stream as
 * qsmd_gen_batch, byte-identical, written to device buffers (hdr_dev[n_hist],
 * events_dev[n_hist * 2 * n_ops], bug_dev nullable) and enqueued on `stream`
 * (NULL = the context's stream) of ctx's device.  Returns 0 or QSMD_ERR_*. */
int qsmd_gen_batch_device(qsmd_ctx* ctx, const qsmd_gen_params* p, uint64_t first, uint64_t n_hist,
                          uint32_t ev_base, qsmd_hdr* hdr_dev, qsmd_event* events_dev,
                          uint8_t* bug_dev, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* QSMD_GEN_H */
