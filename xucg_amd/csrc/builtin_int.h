/*
 * builtin_int.h - state shared by the translation units of libucg_builtin.so's
 * operation engine (not an installed header):
 *   builtin_shm.c   f2, the shared-memory AM transport
 *   builtin_ops.c   f1, the operation engine (slots, stash, steps) and its API
 *   builtin_plan.c  the planner (tree, recursive K-ing, placements)
 *   builtin_rma.c   remote-key steps (device and shared-memory buffers)
 * Internal functions are hidden: the library exports only include/'s API.
 */
#ifndef XUCG_BUILTIN_INT_H
#define XUCG_BUILTIN_INT_H

#include "ucg_builtin_ops.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#define UCG_INTERNAL __attribute__((visibility("hidden")))

/* ======================================================================== */
/* f2: shared-memory AM transport state                                     */
/* ======================================================================== */
typedef struct {
    _Alignas(64) _Atomic uint64_t head;   /* producer index */
    _Alignas(64) _Atomic uint64_t tail;   /* consumer index */
} ring_ctl_t;

typedef struct {
    uint32_t length;    /* payload bytes (without the header) */
    uint32_t reserved;
    uint64_t header;    /* followed by the payload: data = &header */
} cell_t;

#define SEG_HDR_BYTES 128
#define UNEXP_GROUPS  64

/* Per member, after the object's header: who is attached and which op it
 * gave up on (round 6). A peer that stops taking part - its
 * process is gone, or its op ended with an error - must end the ops of the
 * others with a status, never hang them or kill their process. */
typedef struct {
    _Atomic uint64_t pid;       /* the member's process once mapped (0: not yet) */
    uint64_t         pidns;     /* its pid namespace (0: unknown) */
    /* per group slot (group_id % UNEXP_GROUPS): the op this member abandoned
     * last, abandon_word(); 0 = none */
    _Atomic uint64_t abandoned[UNEXP_GROUPS];
} member_ctl_t;

/* an abandoned op: the group's incarnation on this iface, its id and the
 * op's start sequence - the same on every member, since members create
 * groups and start their ops in the same order (a collective's contract) */
static inline uint64_t abandon_word(uint16_t gen, uint16_t group_id, uint64_t seq)
{
    return ((uint64_t)gen << 48) | ((uint64_t)group_id << 32) | (seq & 0xffffffffull);
}

/* Incast cell (the SM-root "bcopy into a shared buffer" of the UCX
 * collectives extension the reference's reducing packers are written for,
 * builtin_pack.c:50-72, 100-148): every child of a root packs the same
 * (header) message into one cell of the root's incast area - the first copies
 * (or, for a concurrent packer, zeroes), the others reduce into it - and the
 * root receives the cell as one message once all `expected` children packed. */
typedef struct {
    _Atomic uint32_t lock;
    _Atomic uint32_t state;     /* INCAST_FREE / _FILLING / _READY */
    _Atomic uint32_t count;     /* children packed so far */
    uint32_t         expected;
    uint32_t         length;    /* payload bytes */
    uint32_t         reserved;
    uint64_t         header;    /* followed by the payload: data = &header */
} incast_cell_t;

enum { INCAST_FREE, INCAST_FILLING, INCAST_READY };

typedef struct {
    _Alignas(64) _Atomic uint64_t ready;   /* cells in INCAST_READY */
} incast_ctl_t;

typedef struct stash {
    struct stash *next;
    uint64_t      header;
    size_t        length;  /* payload bytes */
    uint8_t       data[];
} stash_t;

struct ucg_builtin_shm_iface {
    char      name[256];
    unsigned  members;
    unsigned  my;
    size_t    max_short;
    size_t    cell_size;
    unsigned  cells;
    size_t    ring_bytes;
    size_t    incast_cell_size;
    int       incast_batched;  /* cells hold every child's message side by side */
    size_t    incast_bytes;    /* one member's incast area */
    size_t    incast_base;     /* offset of member 0's incast area */
    size_t    ctl_bytes;       /* header + member_ctl_t[members], rounded to 64 */
    size_t    seg_bytes;
    char     *seg;
    uint64_t  barrier_gen;
    ucs_status_t open_status;  /* why ucg_builtin_shm_iface_open failed */
    /* peer failure (shm_peer_check): the first member found gone, and the
     * status every later barrier and close returns at once (the barrier's
     * count is no longer shared once one member gave up on it). Atomic: the
     * owner's barrier and every group's resend timer thread probe them. */
    _Atomic int      dead;          /* member index + 1, 0 = none found */
    _Atomic int      broken;        /* ucs_status_t; first non-OK one sticks */
    _Atomic uint64_t live_check_ns; /* last liveness probe (monotonic ns) */
    uint16_t  group_gen[UNEXP_GROUPS];  /* groups created per slot */
    /* ops layer: groups by id and messages for groups not created yet
     * (the reference's bctx->group_by_id / bctx->unexpected, builtin.c:
     * 150-205) */
    ucg_builtin_lgroup_t *groups[UNEXP_GROUPS];
    stash_t  *unexpected;
    /* the worker's async context: one recursive lock for every group of this
     * interface (ucg_builtin_lgroup.async_lock points here) */
    pthread_mutex_t async_lock;
};

static inline double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static inline double wait_timeout_s(void)
{
    const char *t = getenv("UCX_BUILTIN_WAIT_TIMEOUT");
    return t ? atof(t) : 300.0;
}

/* how often a waiter that made no progress looks at its peers */
#define PEER_CHECK_S 0.02

/* builtin_shm.c: peer failure. shm_peer_check: the index of a member whose
 * process is gone (probed at most every PEER_CHECK_S; sticky), -1 if none -
 * only called by a member that is idle, so messages a peer sent before it
 * exited are taken in first. shm_abandon / shm_abandoned: publish / read the
 * op a member gave up on (member_ctl_t.abandoned). */
UCG_INTERNAL int      shm_peer_check(ucg_builtin_shm_iface_t *it);
UCG_INTERNAL void     shm_abandon(ucg_builtin_shm_iface_t *it, unsigned slot, uint64_t word);
UCG_INTERNAL uint64_t shm_abandoned(ucg_builtin_shm_iface_t *it, unsigned member,
                                    unsigned slot);

/* ======================================================================== */
/* f1: engine state                                                         */
/* ======================================================================== */
/* builtin/ops/builtin_ops.h:45-60 */
typedef union {
    struct {
        uint16_t group_id;
        union {
            struct {
                uint8_t coll_id;
                uint8_t step_idx;
            };
            uint16_t local_id;
        };
        uint32_t remote_offset;
    };
    uint64_t header;
} ops_header_t;

_Static_assert(sizeof(ops_header_t) == 8, "wire header is 8 bytes");

#define OPS_MAX_STEPS 12

/* the plan methods this engine runs (builtin/plan/builtin_plan.h:28-44), and
 * the aggregation each receive applies (builtin_control.c:960-972) */
typedef enum {
    M_REDUCE_RECURSIVE,   /* send to the step's peers, receive and reduce */
    M_REDUCE_TERMINAL,    /* tree root: receive from every child and reduce */
    M_SEND_TO_SM_ROOT,    /* tree leaf, fan-in (ppn > 2) */
    M_SEND_TERMINAL,      /* tree leaf fan-in at ppn == 2, root fan-out */
    M_RECV_TERMINAL,      /* tree leaf, fan-out: receive the result */
    M_REDUCE_WAYPOINT,    /* receive from the children and reduce, then send
                             the accumulator to the parent */
    M_BCAST_WAYPOINT      /* receive from the parent, then send to the
                             children */
} op_method_t;

typedef enum { AGG_NOP, AGG_REDUCE, AGG_WRITE } op_aggregation_t;

/* bcopy packers of an SM-root child (builtin_pack.c): plain copy, reducing
 * (:50-72) or unsigned-SUM atomic (:100-148) */
typedef enum { PACK_COPY, PACK_REDUCING, PACK_ATOMIC, PACK_BATCHED } op_packer_t;


typedef struct {
    uint8_t     method;           /* op_method_t */
    uint8_t     aggregation;      /* op_aggregation_t */
    uint8_t     step_idx;         /* phase->step_index, 1-based */
    unsigned    send_cnt;         /* endpoints sent to, in this order */
    unsigned    send_peers[UCG_BUILTIN_OPS_MAX_MEMBERS];
    unsigned    recv_cnt;         /* endpoints received from */
    unsigned    recv_peers[UCG_BUILTIN_OPS_MAX_MEMBERS];  /* describe only */
    int         send_recv_buffer; /* 0: send.buffer, 1: recv.buffer */
    int         recv_first;       /* *_WAYPOINT: every receive of the step
                                     before its sends (RECV_BEFORE_SEND1 /
                                     RECV1_BEFORE_SEND, builtin_control.c:
                                     379-389) */
    int         pipelined;        /* a fragmented waypoint: each fragment goes
                                     on once all its contributions are in
                                     (PIPELINED / BY_FRAGMENT_OFFSET,
                                     builtin_control.c:831-834, 978-980) */
    int         incast;           /* sends / receives go through the incast:
                                     1 one reduced message per fragment, 2 (a
                                     root) batched: every child's fragment in
                                     one message, reduced here in order */
    uint8_t     packer;           /* op_packer_t of an incast send */
    unsigned    incast_expected;  /* children packing each incast message */
    size_t      frag_len;         /* 0: single message */
    uint64_t    frags;            /* messages per endpoint */
    uint64_t    fragments_total;  /* recv_cnt x frags */
} op_step_t;

typedef struct {
    ucg_builtin_lcoll_t *req;     /* the op running in this slot */
    uint16_t             expecting;
    stash_t             *msgs;    /* slot->messages */
    stash_t            **msgs_tail; /* &last->next (or &msgs): O(1) append */
} op_slot_t;

struct ucg_builtin_lgroup {
    ucg_builtin_shm_iface_t *iface;
    uint16_t                 group_id;
    unsigned                 size;
    unsigned                 my;
    ucg_builtin_combine_t   *cmb;
    op_slot_t                slots[UCG_BUILTIN_OPS_MAX_CONCURRENT];
    uint8_t                  next_coll_id;
    int                      incast;   /* UCX_BUILTIN_SM_INCAST: 0 n, 1 y, 2 batched */
    uint64_t                 stats[4];
    /* placement and planner knobs (ucg_builtin_lgroup_params_t) */
    uint8_t                  distance[UCG_BUILTIN_OPS_MAX_MEMBERS];
    unsigned                 radix;
    unsigned                 sock_thresh;
    unsigned                 factor;
    /* device buffers of the remote-key steps, registered once per group
     * (the memory registration cache behind ucg_builtin_step_zcopy_prep,
     * builtin_control.c:276-286): an op's buffers return here when it is
     * destroyed and peers' mappings stay open until the group goes, so a key
     * always names the memory it named when it was sent */
    struct rma_pool         *pool;
    unsigned                 npool;
    void                    *arena;           /* device memory made with the group */
    size_t                   arena_bytes, arena_used;
    struct rma_imp          *imp;
    unsigned                 nimp;
    /* the worker's async context (UCS_ASYNC_BLOCK, builtin.c:263-267, 331-335):
     * every entry point holds this recursive lock, and so does the resend
     * timer (builtin.c:284-294, 408-413) when it runs on its own thread. It is
     * the interface's (ucg_builtin_shm_iface.async_lock), as the reference's is
     * the worker's: every group's progress and timer reach the shared rings,
     * the group table and the unexpected list, and deliver each other's
     * messages */
    pthread_mutex_t         *async_lock;
    pthread_cond_t           timer_cv;
    pthread_t                timer;
    int                      timer_on;
    int                      timer_stop;
    double                   timer_tick;
    _Atomic uint64_t         async_resends;
    unsigned                 mem_reg_opt_cnt; /* starts before registering, 0 = never */
    _Atomic uint64_t         async_combines;   /* combines and folds on the timer thread */
    /* peer failure: the group's incarnation on its iface, the ops started so
     * far (an op's sequence number), idle progress calls since the last look
     * at the peers */
    uint16_t                 gen;
    uint64_t                 starts;
    unsigned                 idle_polls;
    double                   peer_check_t;
};

struct ucg_builtin_lcoll {
    ucg_builtin_lgroup_t *g;
    const char  *sbuf;
    char        *rbuf;
    int          count;
    void        *dtype;
    void        *op;
    size_t       dt_len;
    size_t       length;
    const char  *plan;            /* "recursive doubling" / "tree" / ... */
    int          kind;            /* 0 allreduce, 1 reduce */
    char        *scratch;         /* accumulator of a non-root member that
                                     combines in a reduce (rbuf then points
                                     here) */
    unsigned     root;
    int          init_reduce;     /* ucg_builtin_init_reduce on start */
    op_step_t    steps[OPS_MAX_STEPS];
    unsigned     nsteps;
    /* request state (builtin_ops.h:233-241) */
    int          active;
    int          done;            /* set by lcoll_set_done: a waiter polls it unlocked */
    ucs_status_t status;
    uint8_t      coll_id;
    unsigned     cur;
    uint64_t     pending;
    int          step_started;
    int          step_open;       /* a combine step is open */
    int          send_pending;
    int          recv_done;       /* a recv_first step has all its data */
    /* the pipelined waypoint step in progress (builtin_data.c:425-520,
     * builtin_comp_step.inl:155-174) */
    int          pipelining;      /* this step forwards fragment by fragment */
    unsigned    *frag_left;       /* contributions still due per fragment
                                   * (not a byte: a waypoint may have more
                                   * than 255 children) */
    uint64_t    *frag_fifo;       /* complete fragments not yet sent out */
    uint64_t     fifo_head, fifo_tail;
    unsigned     fifo_ep;         /* next endpoint of the head fragment */
    uint64_t     frags_sent;
    uint64_t     pipe_cap;        /* entries of frag_left and frag_fifo */
    unsigned     iter_ep;
    size_t       iter_offset;
    /* device-resident buffers: remote-key steps (the rkey exchange of
     * ucg_builtin_step_create_rkey_bcast and the zero-copy reads of
     * SEND_GET_ZCOPY, builtin_control.c:1014-1076, builtin_data.c:326-340) */
    int          rma;
    char        *rbuf_user;       /* where the result goes; NULL off a
                                     reduce's root */
    void        *dbuf[2];         /* this member's exposed device buffers */
    int          pool_idx[2];     /* their entries in the group's pool */
    uint8_t      key[3][UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
    int          exp_sbuf;        /* send.buffer is registered group memory
                                     (ucg_builtin_lgroup_mem_alloc): exposed in
                                     place as buffer 2, no init copy */
    int          keys_sent;       /* the keys go out on the first start only */
    unsigned     cur_buf;         /* the buffer holding this member's data:
                                     dbuf 0 / 1, or 2 = send.buffer */
    unsigned     readers[3];      /* peers still reading each buffer */
    void        *peer_buf[UCG_BUILTIN_OPS_MAX_MEMBERS][3];
    unsigned     rdy_cnt[OPS_MAX_STEPS];   /* READY messages per step ... */
    uint8_t      rdy_peer[OPS_MAX_STEPS][UCG_BUILTIN_OPS_MAX_MEMBERS];
    uint8_t      rdy_buf[OPS_MAX_STEPS][UCG_BUILTIN_OPS_MAX_MEMBERS];
                                  /* ... in arrival order: the fold order */
    int          rma_sent, rma_recvd, rma_final, rma_busy, rma_again;
    void        *bf_scratch;      /* host one-shot: the butterfly's partial sums */
    size_t       bf_bytes;
    int          oneshot;         /* recursive doubling run as one-shot
                                     reduce-scatter + all-gather (1), or - a
                                     small message - one pass of every member
                                     over all the data (2), or a one-host
                                     tree's fold in one pass (3) */
    /* the memory registration of the recv buffer after MEM_REG_OPT_CNT
     * starts whose steps staged on the device (builtin_control.c:345-373) */
    int          staged_dev;      /* a step of this op staged on the device */
    unsigned     dev_starts;      /* starts since */
    int          rbuf_reg;        /* rbuf registered (dropped in destroy) */
    /* ucg_params_t.completion (api/ucg.h:162-171) */
    int          comp_set;
    ucg_builtin_coll_comp_cb_f comp_cb;
    void        *comp_req;
    size_t       comp_flag_off, comp_status_off;
    struct rma_msg *outbox;       /* control messages not sent yet */
    unsigned     out_head, out_tail, out_cap;
    uint64_t     seq;             /* the group's start count at this start */
    int          peer_ended;      /* finished because of a peer: not published */
};

/* An op may finish on the resend timer's thread while its owner polls `done`
 * outside the lock (lcoll_wait, lcoll_test): the status is written first and
 * published by the release store. */
static inline void lcoll_set_done(ucg_builtin_lcoll_t *c)
{
    __atomic_store_n(&c->done, 1, __ATOMIC_RELEASE);
}

static inline int lcoll_is_done(const ucg_builtin_lcoll_t *c)
{
    return __atomic_load_n(&c->done, __ATOMIC_ACQUIRE);
}

/* planner state (builtin_plan.c) */
#define TREE_MAX_RADIX 128   /* UCG_BUILTIN_TREE_MAX_RADIX, builtin_plan.h:98 */
#define PM               UCG_BUILTIN_OPS_MAX_MEMBERS

typedef struct {
    unsigned n, my;              /* group size, my virtual index */
    uint8_t  d[PM];               /* my distances, virtual order */
    unsigned v2r[PM];
    unsigned radix, sock_thresh, factor;
} plan_ctx_t;

enum {
    D_SELF = UCG_BUILTIN_DISTANCE_SELF, D_SOCKET = UCG_BUILTIN_DISTANCE_SOCKET,
    D_HOST = UCG_BUILTIN_DISTANCE_HOST, D_NET = UCG_BUILTIN_DISTANCE_NET,
    D_LAST = 255                 /* UCG_GROUP_MEMBER_DISTANCE_LAST */
};

#define RMA_DEV 1       /* device buffers: HIP IPC keys, kernels */
#define RMA_SHM 2       /* host buffers: POSIX shared memory keys, reduce_cb_f */

/* builtin_ops.c */
UCG_INTERNAL size_t parse_memunits(const char *s, size_t dflt);   /* builtin_combine.c */
UCG_INTERNAL void finish(ucg_builtin_lcoll_t *c, ucs_status_t status);
UCG_INTERNAL int ops_on_timer_thread(void);     /* the resend timer's thread */
UCG_INTERNAL void rma_group_init(ucg_builtin_lgroup_t *g);
UCG_INTERNAL void lcoll_notify(ucg_builtin_lcoll_t *c);

/* builtin_plan.c */
UCG_INTERNAL ucs_status_t plan_ctx_init(ucg_builtin_lgroup_t *g, unsigned root,
                                        plan_ctx_t *pc);
UCG_INTERNAL ucs_status_t plan_tree(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc,
                                    int fanout, unsigned *ppn);
UCG_INTERNAL ucs_status_t plan_recursive(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc,
                                         unsigned *ppn_out);
UCG_INTERNAL ucs_status_t plan_finish(ucg_builtin_lcoll_t *c, unsigned ppn);

/* builtin_rma.c */
UCG_INTERNAL int          rma_kind(ucg_builtin_lgroup_t *g, const void *sbuf,
                                   const void *rbuf, size_t length);
UCG_INTERNAL ucs_status_t rma_setup(ucg_builtin_lcoll_t *c, void *rbuf_user);
UCG_INTERNAL ucs_status_t rma_start(ucg_builtin_lcoll_t *c, op_slot_t *slot);
UCG_INTERNAL void         rma_msg(ucg_builtin_lcoll_t *c, ops_header_t h,
                                  const void *data, size_t length);
UCG_INTERNAL void         rma_advance(ucg_builtin_lcoll_t *c);
UCG_INTERNAL void         rma_free(ucg_builtin_lcoll_t *c);
UCG_INTERNAL void         rma_group_free(ucg_builtin_lgroup_t *g);

#endif
