/*
 * builtin_ops.c - the builtin planner's operation engine around the combine
 * and a minimal shared-memory AM transport (include/ucg_builtin_ops.h).
 *
 * This is a C restatement of the receive/step machinery of the reference's
 * builtin/ops for the REDUCE_RECURSIVE method (see the header for file:line
 * anchors), written against this build's combine dispatcher instead of a
 * direct reduce_cb_f call. It is what lets the reference's allreduce plan run
 * end to end between processes with no UCX underneath.
 */
#define _GNU_SOURCE
#include "ucg_builtin_ops.h"

#include <fcntl.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

/* ======================================================================== */
/* f2: shared-memory AM transport                                           */
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

#define SEG_CTL_BYTES 128
#define UNEXP_GROUPS  64

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
    size_t    incast_bytes;    /* one member's incast area */
    size_t    incast_base;     /* offset of member 0's incast area */
    size_t    seg_bytes;
    char     *seg;
    uint64_t  barrier_gen;
    /* ops layer: groups by id and messages for groups not created yet
     * (the reference's bctx->group_by_id / bctx->unexpected, builtin.c:
     * 150-205) */
    ucg_builtin_lgroup_t *groups[UNEXP_GROUPS];
    stash_t  *unexpected;
};

static ring_ctl_t *ring_ctl(ucg_builtin_shm_iface_t *it, unsigned src, unsigned dst)
{
    return (ring_ctl_t*)(it->seg + SEG_CTL_BYTES +
                         ((size_t)src * it->members + dst) * it->ring_bytes);
}

static cell_t *ring_cell(ucg_builtin_shm_iface_t *it, ring_ctl_t *r, uint64_t idx)
{
    return (cell_t*)((char*)r + sizeof(ring_ctl_t) + (idx % it->cells) * it->cell_size);
}

static incast_ctl_t *incast_ctl(ucg_builtin_shm_iface_t *it, unsigned member)
{
    return (incast_ctl_t*)(it->seg + it->incast_base + member * it->incast_bytes);
}

static incast_cell_t *incast_cell(ucg_builtin_shm_iface_t *it, unsigned member,
                                  unsigned idx)
{
    return (incast_cell_t*)((char*)incast_ctl(it, member) + sizeof(incast_ctl_t) +
                            (size_t)idx * it->incast_cell_size);
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double wait_timeout_s(void)
{
    const char *t = getenv("UCX_BUILTIN_WAIT_TIMEOUT");
    return t ? atof(t) : 300.0;
}

ucs_status_t ucg_builtin_shm_iface_open(const char *name, unsigned members,
                                        unsigned my_index, size_t max_short,
                                        unsigned ring_cells,
                                        ucg_builtin_shm_iface_t **iface_p)
{
    ucg_builtin_shm_iface_t *it;
    int fd;
    struct stat stt;

    if (name == NULL || iface_p == NULL || members == 0 ||
        members > UCG_BUILTIN_OPS_MAX_MEMBERS || my_index >= members ||
        max_short <= 8 || max_short > (1u << 20) || ring_cells < 2) {
        return UCS_ERR_INVALID_PARAM;
    }
    it = calloc(1, sizeof(*it));
    if (it == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    snprintf(it->name, sizeof(it->name), "/%s", name[0] == '/' ? name + 1 : name);
    it->members    = members;
    it->my         = my_index;
    it->max_short  = max_short;
    it->cells      = ring_cells;
    it->cell_size  = (sizeof(cell_t) + (max_short - 8) + 63) & ~(size_t)63;
    it->ring_bytes = sizeof(ring_ctl_t) + (size_t)ring_cells * it->cell_size;
    it->incast_cell_size = (sizeof(incast_cell_t) + (max_short - 8) + 63) & ~(size_t)63;
    it->incast_bytes     = sizeof(incast_ctl_t) + (size_t)ring_cells * it->incast_cell_size;
    it->incast_base      = SEG_CTL_BYTES + (size_t)members * members * it->ring_bytes;
    it->seg_bytes        = it->incast_base + (size_t)members * it->incast_bytes;

    fd = shm_open(it->name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        free(it);
        return UCS_ERR_IO_ERROR;
    }
    /* a fresh object is zero-filled: every ring starts empty (head = tail) */
    if (fstat(fd, &stt) != 0 ||
        ((size_t)stt.st_size < it->seg_bytes && ftruncate(fd, it->seg_bytes) != 0)) {
        close(fd);
        free(it);
        return UCS_ERR_IO_ERROR;
    }
    it->seg = mmap(NULL, it->seg_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (it->seg == MAP_FAILED) {
        free(it);
        return UCS_ERR_NO_MEMORY;
    }
    ucg_builtin_shm_barrier(it);   /* everybody mapped before any send */
    *iface_p = it;
    return UCS_OK;
}

void ucg_builtin_shm_iface_close(ucg_builtin_shm_iface_t *it)
{
    stash_t *m;
    if (it == NULL) {
        return;
    }
    ucg_builtin_shm_barrier(it);
    munmap(it->seg, it->seg_bytes);
    if (it->my == 0) {
        shm_unlink(it->name);
    }
    while ((m = it->unexpected) != NULL) {
        it->unexpected = m->next;
        free(m);
    }
    free(it);
}

size_t ucg_builtin_shm_iface_max_short(ucg_builtin_shm_iface_t *it)
{
    return it ? it->max_short : 0;
}

void ucg_builtin_shm_barrier(ucg_builtin_shm_iface_t *it)
{
    _Atomic uint64_t *arrive = (_Atomic uint64_t*)it->seg;
    uint64_t gen = ++it->barrier_gen;
    double t0 = now_s(), lim = wait_timeout_s();
    atomic_fetch_add_explicit(arrive, 1, memory_order_acq_rel);
    while (atomic_load_explicit(arrive, memory_order_acquire) < gen * it->members) {
        if (now_s() - t0 > lim) {
            fprintf(stderr, "ucg_builtin_shm_barrier(%s): timed out after %.0f s\n",
                    it->name, lim);
            abort();
        }
        sched_yield();
    }
}

ucs_status_t ucg_builtin_shm_am_short(ucg_builtin_shm_iface_t *it, unsigned peer,
                                      uint64_t header, const void *payload,
                                      size_t length)
{
    ring_ctl_t *r;
    uint64_t head, tail;
    cell_t *c;

    if (peer >= it->members || peer == it->my) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (length + 8 > it->max_short) {
        return UCS_ERR_INVALID_PARAM;   /* UCS_ERR_MESSAGE_TRUNCATED in UCT */
    }
    r    = ring_ctl(it, it->my, peer);
    head = atomic_load_explicit(&r->head, memory_order_relaxed);
    tail = atomic_load_explicit(&r->tail, memory_order_acquire);
    if (head - tail >= it->cells) {
        return UCS_ERR_NO_RESOURCE;
    }
    c = ring_cell(it, r, head);
    c->length = (uint32_t)length;
    c->header = header;
    if (length) {
        memcpy(c + 1, payload, length);
    }
    atomic_store_explicit(&r->head, head + 1, memory_order_release);
    return UCS_OK;
}

static void spin_lock(_Atomic uint32_t *l)
{
    unsigned spins = 0;
    uint32_t z = 0;
    double t0 = 0.0;
    while (!atomic_compare_exchange_weak_explicit(l, &z, 1, memory_order_acquire,
                                                  memory_order_relaxed)) {
        z = 0;
        /* the holder packs at most one fragment: spin briefly, then yield;
         * a holder that never lets go (a dead peer) is fatal, not a hang */
        if (++spins < 256) {
            __builtin_ia32_pause();
            continue;
        }
        if (t0 == 0.0) {
            t0 = now_s();
        } else if ((spins & 1023) == 0 && now_s() - t0 > wait_timeout_s()) {
            fprintf(stderr, "ucg_builtin_shm: incast cell lock held for over %.0f s\n",
                    wait_timeout_s());
            abort();
        }
        sched_yield();
    }
}

static void spin_unlock(_Atomic uint32_t *l)
{
    atomic_store_explicit(l, 0, memory_order_release);
}

ucs_status_t ucg_builtin_shm_am_incast(ucg_builtin_shm_iface_t *it, unsigned root,
                                       uint64_t header, unsigned expected,
                                       size_t length, ucg_builtin_pack_cb_f pack,
                                       void *arg, int concurrent)
{
    unsigned idx;
    incast_cell_t *c;
    int first;

    if (root >= it->members || root == it->my || expected == 0 || pack == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (length + 8 > it->max_short) {
        return UCS_ERR_INVALID_PARAM;
    }
    /* the cell of this message: consecutive fragments of one message
     * (remote_offset in steps of at most max_short - 8) take consecutive
     * cells from a start that a multiplicative hash of the rest of the
     * header (group, coll_id, step) spreads out */
    idx = (unsigned)((((header & 0xffffffffull) * 0x9E3779B97F4A7C15ull) >> 40) +
                     (header >> 32) / (it->max_short - 8)) % it->cells;
    c   = incast_cell(it, root, idx);
    spin_lock(&c->lock);
    /* acquire: the root's reads of a delivered cell precede our writes */
    if (atomic_load_explicit(&c->state, memory_order_acquire) == INCAST_FREE) {
        atomic_store_explicit(&c->state, INCAST_FILLING, memory_order_relaxed);
        atomic_store_explicit(&c->count, 0, memory_order_relaxed);
        c->header   = header;
        c->expected = expected;
        c->length   = (uint32_t)length;
        first       = 1;
    } else if (atomic_load_explicit(&c->state, memory_order_acquire) == INCAST_FILLING &&
               c->header == header) {
        first = 0;
    } else {
        spin_unlock(&c->lock);
        return UCS_ERR_NO_RESOURCE;   /* cell busy with another message */
    }
    if (concurrent) {
        /* atomic packers add into a zeroed cell outside the lock */
        if (first) {
            memset(c + 1, 0, length);
        }
        spin_unlock(&c->lock);
        pack(arg, c + 1, 1);
    } else {
        pack(arg, c + 1, !first);     /* first copies, the others reduce */
    }
    if (atomic_fetch_add_explicit(&c->count, 1, memory_order_acq_rel) + 1 == expected) {
        atomic_store_explicit(&c->state, INCAST_READY, memory_order_release);
        atomic_fetch_add_explicit(&incast_ctl(it, root)->ready, 1, memory_order_release);
    }
    if (!concurrent) {
        spin_unlock(&c->lock);
    }
    return UCS_OK;
}

static unsigned incast_progress(ucg_builtin_shm_iface_t *it, ucg_builtin_am_cb_f cb,
                                void *arg)
{
    incast_ctl_t *ctl = incast_ctl(it, it->my);
    unsigned i, n = 0;
    if (atomic_load_explicit(&ctl->ready, memory_order_acquire) == 0) {
        return 0;
    }
    for (i = 0; i < it->cells; i++) {
        incast_cell_t *c = incast_cell(it, it->my, i);
        if (atomic_load_explicit(&c->state, memory_order_acquire) != INCAST_READY) {
            continue;
        }
        (void)cb(arg, &c->header, 8 + (size_t)c->length);
        atomic_fetch_sub_explicit(&ctl->ready, 1, memory_order_relaxed);
        atomic_store_explicit(&c->state, INCAST_FREE, memory_order_release);
        n++;
    }
    return n;
}

unsigned ucg_builtin_shm_progress(ucg_builtin_shm_iface_t *it,
                                  ucg_builtin_am_cb_f cb, void *arg)
{
    unsigned src, n = incast_progress(it, cb, arg);
    for (src = 0; src < it->members; src++) {
        ring_ctl_t *r;
        uint64_t tail, head;
        if (src == it->my) {
            continue;
        }
        r    = ring_ctl(it, src, it->my);
        tail = atomic_load_explicit(&r->tail, memory_order_relaxed);
        head = atomic_load_explicit(&r->head, memory_order_acquire);
        while (tail < head) {
            cell_t *c = ring_cell(it, r, tail);
            (void)cb(arg, &c->header, 8 + (size_t)c->length);
            tail++;
            /* the cell is free only after the callback returned */
            atomic_store_explicit(&r->tail, tail, memory_order_release);
            n++;
        }
    }
    return n;
}

/* ======================================================================== */
/* f1: the builtin operation engine                                         */
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
typedef enum { PACK_COPY, PACK_REDUCING, PACK_ATOMIC } op_packer_t;
static const char *const packer_name[] = {"copy", "reducing", "atomic"};

static const char *const method_name[] = {
    "REDUCE_RECURSIVE", "REDUCE_TERMINAL", "SEND_TO_SM_ROOT", "SEND_TERMINAL",
    "RECV_TERMINAL", "REDUCE_WAYPOINT", "BCAST_WAYPOINT"
};

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
    int         incast;           /* sends / receives go through the incast */
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
    int                      incast;   /* UCX_BUILTIN_SM_INCAST */
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
    struct rma_imp          *imp;
    unsigned                 nimp;
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
    int          done;
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
    uint8_t      key[2][UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
    int          keys_sent;       /* the keys go out on the first start only */
    unsigned     cur_buf;         /* the dbuf holding this member's data */
    unsigned     readers[2];      /* peers still reading each dbuf */
    void        *peer_buf[UCG_BUILTIN_OPS_MAX_MEMBERS][2];
    unsigned     rdy_cnt[OPS_MAX_STEPS];   /* READY messages per step ... */
    uint8_t      rdy_peer[OPS_MAX_STEPS][UCG_BUILTIN_OPS_MAX_MEMBERS];
    uint8_t      rdy_buf[OPS_MAX_STEPS][UCG_BUILTIN_OPS_MAX_MEMBERS];
                                  /* ... in arrival order: the fold order */
    int          rma_sent, rma_recvd, rma_final, rma_busy, rma_again;
    struct rma_msg *outbox;       /* control messages not sent yet */
    unsigned     out_head, out_tail, out_cap;
};

static int  recv_cb(ucg_builtin_lcoll_t *c, uint64_t offset, const void *data,
                    size_t length);
static void step_execute(ucg_builtin_lcoll_t *c);
static void rma_msg(ucg_builtin_lcoll_t *c, ops_header_t h, const void *data,
                    size_t length);
static void rma_advance(ucg_builtin_lcoll_t *c);
static void rma_group_free(ucg_builtin_lgroup_t *g);

static stash_t *stash_new(uint64_t header, const void *payload, size_t length)
{
    stash_t *m = malloc(sizeof(*m) + length);
    if (m) {
        m->next   = NULL;
        m->header = header;
        m->length = length;
        memcpy(m->data, payload, length);
    }
    return m;
}

static void stash_append(stash_t **list, stash_t *m)
{
    while (*list) {
        list = &(*list)->next;
    }
    *list = m;
}

/* a slot's stash is appended to on every early message: keep it O(1) */
static void slot_stash(op_slot_t *slot, stash_t *m)
{
    *slot->msgs_tail = m;
    slot->msgs_tail  = &m->next;
}

/* finish the op: ucg_builtin_comp_last_step_cb, builtin_comp_step.inl:8-38 */
static void finish(ucg_builtin_lcoll_t *c, ucs_status_t status)
{
    op_slot_t *slot = &c->g->slots[c->coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT];
    if (c->step_open) {
        ucs_status_t st = ucg_builtin_combine_step_end(c->g->cmb);
        if (status == UCS_OK) {
            status = st;
        }
        c->step_open = 0;
    }
    c->status       = status;
    c->done         = 1;
    c->active       = 0;
    c->send_pending = 0;
    c->step_started = 0;
    slot->req       = NULL;
    slot->expecting = 0;
}

/* ucg_builtin_step_check_pending, builtin_comp_step.inl:403-462 */
static void check_pending(ucg_builtin_lcoll_t *c, uint16_t local_id)
{
    op_slot_t *slot = &c->g->slots[c->coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT];
    stash_t **pp = &slot->msgs, *m;
    slot->expecting = local_id;
    for (;;) {
        /* the messages before pp did not match and still do not: a step
         * that is not done yet only sends from recv_cb, so the list is not
         * touched behind the cursor */
        while (*pp) {
            ops_header_t h;
            h.header = (*pp)->header;
            if (h.local_id == local_id) {
                break;
            }
            pp = &(*pp)->next;
        }
        if ((m = *pp) == NULL) {
            return;
        }
        *pp = m->next;   /* remove first: the next call may recurse here */
        if (m->next == NULL) {
            slot->msgs_tail = pp;
        }
        ops_header_t h;
        h.header = m->header;
        int step_done = recv_cb(c, h.remote_offset, m->data, m->length);
        free(m);
        if (step_done) {
            return;      /* the next step (if any) drained its own messages */
        }
    }
}

/* ucg_builtin_comp_step_cb / ucg_builtin_comp_last_step_cb,
 * builtin_comp_step.inl:8-95: close the step's combine (the device mirror goes
 * back to recv_buffer before the next step sends it, builtin_control.c:
 * 850-857), then move on */
static void step_complete(ucg_builtin_lcoll_t *c)
{
    if (c->step_open) {
        ucs_status_t st = ucg_builtin_combine_step_end(c->g->cmb);
        c->step_open = 0;
        if (st != UCS_OK) {
            finish(c, st);
            return;
        }
    }
    c->step_started = 0;
    if (c->cur + 1 == c->nsteps) {
        finish(c, UCS_OK);
    } else {
        c->cur++;
        step_execute(c);
    }
}

typedef struct {
    ucg_builtin_lcoll_t *c;
    const char          *src;
    size_t               length;
    ucs_status_t         status;
} pack_arg_t;

/* UCG_BUILTIN_REDUCING_PACK_CB, builtin_pack.c:50-72: the first child's data
 * is copied, every later child's is reduced into the transport buffer,
 * dst = mine (op) dst, through ucg_builtin_atomic_reduce_part (:22-28) - here
 * the combine dispatcher (device for large classified fragments). */
static void pack_reducing(void *arg, void *dest, int reducing)
{
    pack_arg_t *a = arg;
    ucg_builtin_lcoll_t *c = a->c;
    if (!reducing) {
        memcpy(dest, a->src, a->length);
        return;
    }
    a->status = ucg_builtin_combine_reduce(c->g->cmb, c->op, (void*)a->src, dest,
                                           (int)(a->length / c->dt_len), c->dtype);
}

/* UCG_BUILTIN_ATOMIC_{SINGLE,MULTIPLE}_PACK_CB, builtin_pack.c:100-148, for
 * unsigned-integer SUM: ucs_atomic_add of each element into the zeroed cell.
 * Unlike the reference's "multiple" packer (which adds send_buffer[0] to every
 * element, :119-122) element i adds element i. */
static void pack_atomic(void *arg, void *dest, int reducing)
{
    pack_arg_t *a = arg;
    size_t i, n = a->length / a->c->dt_len;
    (void)reducing;
#define ADD_ALL(T)                                                            \
    for (i = 0; i < n; i++) {                                                 \
        T v;                                                                  \
        memcpy(&v, a->src + i * sizeof(T), sizeof(T));                        \
        __atomic_fetch_add((T*)dest + i, v, __ATOMIC_RELAXED);                \
    }
    switch (a->c->dt_len) {
    case 1: ADD_ALL(uint8_t);  break;
    case 2: ADD_ALL(uint16_t); break;
    case 4: ADD_ALL(uint32_t); break;
    case 8: ADD_ALL(uint64_t); break;
    default: a->status = UCS_ERR_UNSUPPORTED; break;
    }
#undef ADD_ALL
}

/* one message of a step to one endpoint: uct_ep_am_short, or the incast
 * bcopy with the step's packer */
static ucs_status_t send_one(ucg_builtin_lcoll_t *c, const op_step_t *s,
                             unsigned peer, uint64_t header, const char *buf,
                             size_t n)
{
    pack_arg_t a;
    ucs_status_t st;
    if (!s->incast) {
        return ucg_builtin_shm_am_short(c->g->iface, peer, header, buf, n);
    }
    a.c = c;
    a.src = buf;
    a.length = n;
    a.status = UCS_OK;
    st = ucg_builtin_shm_am_incast(c->g->iface, peer, header, s->incast_expected, n,
                                   s->packer == PACK_ATOMIC ? pack_atomic : pack_reducing,
                                   &a, s->packer == PACK_ATOMIC);
    return (st == UCS_OK) ? a.status : st;
}

/* the send half of a step: every fragment to every endpoint of the step
 * (endpoint-major, resumable at iter_ep / iter_offset after
 * UCS_ERR_NO_RESOURCE, builtin_data.c:470-517 and ucg_builtin_step_
 * am_short_max :83-137). Returns 1 when every message went out, 0 when it
 * has to be resumed (send_pending) or the op failed. */
static int step_send(ucg_builtin_lcoll_t *c)
{
    ucg_builtin_lgroup_t *g = c->g;
    op_step_t *s = &c->steps[c->cur];
    const char *sbuf = s->send_recv_buffer ? c->rbuf : c->sbuf;
    ops_header_t h;
    ucs_status_t st;

    h.header   = 0;
    h.group_id = g->group_id;
    h.coll_id  = c->coll_id;
    h.step_idx = s->step_idx;
    for (; c->iter_ep < s->send_cnt; c->iter_ep++) {
        unsigned peer = s->send_peers[c->iter_ep];
        if (s->frag_len == 0) {
            if (c->iter_offset == 0) {
                h.remote_offset = 0;
                st = send_one(c, s, peer, h.header, sbuf, c->length);
                if (st == UCS_ERR_NO_RESOURCE) {
                    c->send_pending = 1;  /* ucg_builtin_req_enqueue_resend */
                    return 0;
                }
                if (st != UCS_OK) {
                    finish(c, st);
                    return 0;
                }
                g->stats[0]++;
            }
        } else {
            while (c->iter_offset < c->length) {
                size_t n = c->length - c->iter_offset;
                if (n > s->frag_len) {
                    n = s->frag_len;
                }
                h.remote_offset = (uint32_t)c->iter_offset;
                st = send_one(c, s, peer, h.header, sbuf + c->iter_offset, n);
                if (st == UCS_ERR_NO_RESOURCE) {
                    c->send_pending = 1;
                    return 0;
                }
                if (st != UCS_OK) {
                    finish(c, st);
                    return 0;
                }
                g->stats[0]++;
                c->iter_offset += n;
            }
        }
        c->iter_offset = 0;   /* next endpoint starts from the first byte */
    }
    c->send_pending = 0;
    return 1;
}

/* the sends of a pipelined waypoint: every fragment whose contributions are
 * all in, to every endpoint of the step, oldest first, resumable after
 * UCS_ERR_NO_RESOURCE at (fifo_head, fifo_ep) - the reference marks such a
 * fragment FRAG_PENDING and resends it (builtin_data.c:496-520, 650-657).
 * Returns 1 when nothing is left to send for now, 0 when it has to be
 * resumed or the op failed. */
static int pipe_send(ucg_builtin_lcoll_t *c)
{
    ucg_builtin_lgroup_t *g = c->g;
    op_step_t *s = &c->steps[c->cur];
    ops_header_t h;
    ucs_status_t st;

    h.header   = 0;
    h.group_id = g->group_id;
    h.coll_id  = c->coll_id;
    h.step_idx = s->step_idx;
    while (c->fifo_head != c->fifo_tail) {
        const uint64_t idx = c->frag_fifo[c->fifo_head % c->pipe_cap];
        const size_t off   = (size_t)idx * s->frag_len;
        const size_t n     = c->length - off < s->frag_len ? c->length - off : s->frag_len;
        h.remote_offset    = (uint32_t)off;
        for (; c->fifo_ep < s->send_cnt; c->fifo_ep++) {
            st = send_one(c, s, s->send_peers[c->fifo_ep], h.header, c->rbuf + off, n);
            if (st == UCS_ERR_NO_RESOURCE) {
                c->send_pending = 1;
                return 0;
            }
            if (st != UCS_OK) {
                finish(c, st);
                return 0;
            }
            g->stats[0]++;
        }
        c->fifo_ep = 0;
        c->fifo_head++;
        c->frags_sent++;
    }
    c->send_pending = 0;
    return 1;
}

/* ucg_builtin_step_execute, builtin_data.c:411-668. A step sends first and
 * then either completes (no receive: comp_criteria SEND, builtin_control.c:
 * 1000-1002) or drains what is already stashed for it (builtin_comp_step.inl:
 * 403-462). A *_WAYPOINT step (recv_first) receives first - from its
 * children, reducing, or from its parent - and sends once the data is
 * complete (comp_action SEND, builtin_control.c:1003-1007): recv_cb comes
 * back here with recv_done set. */
static void step_execute(ucg_builtin_lcoll_t *c)
{
    ucg_builtin_lgroup_t *g = c->g;
    op_step_t *s = &c->steps[c->cur];
    ops_header_t h;
    ucs_status_t st;

    if (!c->step_started) {
        if (s->aggregation == AGG_REDUCE) {
            st = ucg_builtin_combine_step_begin(g->cmb, c->op, c->dtype, c->rbuf,
                                                c->length);
            if (st == UCS_OK) {
                c->step_open = 1;
            } else if (st != UCS_ERR_BUSY) {
                finish(c, st);
                return;
            }
            /* UCS_ERR_BUSY: another op of this group holds the step staging;
             * this step combines each fragment on its own (recv_cb) */
        }
        c->step_started = 1;
        c->recv_done    = 0;
        c->pending      = s->fragments_total;
        c->iter_ep      = 0;
        c->iter_offset  = 0;
        /* fragment by fragment only while each fragment is combined into
         * recv.buffer as it arrives: a step mirrored on the device holds its
         * data until step_end */
        c->pipelining   = s->pipelined &&
                          !(c->step_open && ucg_builtin_combine_step_on_device(g->cmb));
        if (c->pipelining) {
            uint64_t f;
            for (f = 0; f < s->frags; f++) {
                c->frag_left[f] = s->recv_cnt;
            }
            c->fifo_head  = c->fifo_tail = 0;
            c->fifo_ep    = 0;
            c->frags_sent = 0;
        }
    }
    h.header   = 0;
    h.group_id = g->group_id;
    h.coll_id  = c->coll_id;
    h.step_idx = s->step_idx;
    if (c->pipelining) {
        if (!pipe_send(c)) {
            return;
        }
        if (c->recv_done && c->frags_sent == s->frags) {
            step_complete(c);
            return;
        }
        if (!c->recv_done) {
            check_pending(c, h.local_id);
        }
        return;
    }
    if (s->recv_first && !c->recv_done) {
        check_pending(c, h.local_id);
        return;
    }
    if (!step_send(c)) {
        return;
    }
    if (s->recv_first || s->recv_cnt == 0) {
        step_complete(c);
        return;
    }
    check_pending(c, h.local_id);
}

/* ucg_builtin_step_recv_cb -> recv_handle_chunk + handle_comp,
 * builtin_comp_step.inl:184-232, 314-401; returns 1 when the step's receives
 * are done */
static int recv_cb(ucg_builtin_lcoll_t *c, uint64_t offset, const void *data,
                   size_t length)
{
    op_step_t *s = &c->steps[c->cur];
    ucs_status_t st = UCS_OK;

    if (offset + length > c->length) {
        st = UCS_ERR_IO_ERROR;          /* a message outside recv.buffer */
    } else if (s->aggregation == AGG_REDUCE) {
        st = c->step_open ?
             ucg_builtin_combine_fragment(c->g->cmb, offset, data, length) :
             /* ucg_builtin_mpi_reduce_fragment, builtin_comp_step.inl:112-120 */
             ucg_builtin_combine_reduce(c->g->cmb, c->op, (void*)data,
                                        c->rbuf + offset, (int)(length / c->dt_len),
                                        c->dtype);
    } else if (s->aggregation == AGG_WRITE) {
        memcpy(c->rbuf + offset, data, length);   /* :204-210 */
    }
    if (st != UCS_OK) {
        finish(c, st);      /* recv_handle_error, :332-333 */
        return 1;
    }
    if (c->pipelining) {
        /* ucg_builtin_comp_send_check_frag_by_offset, :155-174: the
         * fragment at this offset is complete once every contributor's part
         * of it was combined; it goes on at once */
        const uint64_t idx = offset / s->frag_len;
        if (--c->frag_left[idx] == 0) {
            c->frag_fifo[c->fifo_tail++ % c->pipe_cap] = idx;
        }
        if (--c->pending == 0) {
            c->recv_done = 1;
        }
        if (!pipe_send(c)) {
            return c->recv_done || c->done;   /* resumed by the resend path */
        }
        if (c->recv_done && c->frags_sent == s->frags) {
            step_complete(c);
            return 1;
        }
        return c->recv_done;
    }
    if (--c->pending != 0) {
        return 0;
    }
    if (s->recv_first) {
        /* the accumulator goes out next: its device mirror back to
         * recv.buffer first, as before any send of it */
        if (c->step_open) {
            st = ucg_builtin_combine_step_end(c->g->cmb);
            c->step_open = 0;
            if (st != UCS_OK) {
                finish(c, st);
                return 1;
            }
        }
        c->recv_done = 1;
        step_execute(c);
        return 1;
    }
    step_complete(c);
    return 1;
}

/* ucg_builtin_am_handler, builtin/builtin.c:133-219 */
static ucs_status_t am_handler(void *arg, void *data, size_t length)
{
    ucg_builtin_shm_iface_t *it = arg;
    ops_header_t h;
    ucg_builtin_lgroup_t *g;
    op_slot_t *slot;
    stash_t *m;

    memcpy(&h.header, data, 8);
    g = it->groups[h.group_id % UNEXP_GROUPS];
    if (g == NULL || g->group_id != h.group_id) {
        m = stash_new(h.header, (char*)data + 8, length - 8);
        if (m) {
            stash_append(&it->unexpected, m);
        }
        return UCS_OK;
    }
    slot = &g->slots[h.coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT];
    if (slot->req && slot->req->rma && h.coll_id == slot->req->coll_id) {
        g->stats[1]++;
        rma_msg(slot->req, h, (char*)data + 8, length - 8);
        return UCS_OK;
    }
    if (slot->req && h.local_id == slot->expecting) {
        g->stats[1]++;
        (void)recv_cb(slot->req, h.remote_offset, (char*)data + 8, length - 8);
        return UCS_OK;
    }
    g->stats[2]++;
    m = stash_new(h.header, (char*)data + 8, length - 8);
    if (m == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    slot_stash(slot, m);
    return UCS_OK;
}

static unsigned env_uint(const char *name, unsigned dflt)
{
    const char *e = getenv(name);
    return (e && *e) ? (unsigned)strtoul(e, NULL, 0) : dflt;
}

ucs_status_t ucg_builtin_lgroup_create_ex(ucg_builtin_shm_iface_t *iface,
                                          uint16_t group_id, unsigned member_count,
                                          unsigned my_index,
                                          ucg_builtin_combine_t *combine,
                                          const ucg_builtin_lgroup_params_t *params,
                                          ucg_builtin_lgroup_t **group_p)
{
    ucg_builtin_lgroup_t *g;
    stash_t **pp;
    unsigned m;

    if (iface == NULL || group_p == NULL || combine == NULL || group_id == 0 ||
        member_count != iface->members || my_index != iface->my) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (params && params->distance) {
        for (m = 0; m < member_count; m++) {
            /* distance[my] = SELF and no other member at SELF; FAULT and
             * LAST are not placements */
            if ((params->distance[m] == UCG_BUILTIN_DISTANCE_SELF) != (m == my_index) ||
                params->distance[m] > UCG_BUILTIN_DISTANCE_NET) {
                return UCS_ERR_INVALID_PARAM;
            }
        }
    }
    if (iface->groups[group_id % UNEXP_GROUPS] != NULL) {
        return UCS_ERR_BUSY;
    }
    g = calloc(1, sizeof(*g));
    if (g == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    g->iface    = iface;
    g->group_id = group_id;
    g->size     = member_count;
    g->my       = my_index;
    g->cmb      = combine;
    {
        const char *e = getenv("UCX_BUILTIN_SM_INCAST");
        g->incast = e && (e[0] == 'y' || e[0] == 'Y' || e[0] == '1');
    }
    for (m = 0; m < UCG_BUILTIN_OPS_MAX_CONCURRENT; m++) {
        g->slots[m].msgs_tail = &g->slots[m].msgs;
    }
    for (m = 0; m < member_count; m++) {
        g->distance[m] = (params && params->distance) ? params->distance[m] :
                         (m == my_index) ? UCG_BUILTIN_DISTANCE_SELF : UCG_BUILTIN_DISTANCE_HOST;
    }
    /* builtin/plan/builtin_tree.c:18-29, builtin_recursive.c:13-18 */
    g->radix       = (params && params->tree_radix) ? params->tree_radix :
                     env_uint("UCX_BUILTIN_TREE_RADIX", 8);
    g->sock_thresh = (params && params->sock_thresh) ? params->sock_thresh :
                     env_uint("UCX_BUILTIN_TREE_SOCKET_LEVEL_PPN_THRESH", 16);
    g->factor      = (params && params->recursive_factor) ? params->recursive_factor :
                     env_uint("UCX_BUILTIN_RECURSIVE_FACTOR", 2);
    iface->groups[group_id % UNEXP_GROUPS] = g;
    /* adopt messages that arrived before the group existed (builtin.c:
     * 424-446) */
    pp = &iface->unexpected;
    while (*pp) {
        ops_header_t h;
        h.header = (*pp)->header;
        if (h.group_id == group_id) {
            stash_t *msg = *pp;
            *pp = msg->next;
            msg->next = NULL;
            slot_stash(&g->slots[h.coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT], msg);
        } else {
            pp = &(*pp)->next;
        }
    }
    *group_p = g;
    return UCS_OK;
}

ucs_status_t ucg_builtin_lgroup_create(ucg_builtin_shm_iface_t *iface,
                                       uint16_t group_id, unsigned member_count,
                                       unsigned my_index,
                                       ucg_builtin_combine_t *combine,
                                       ucg_builtin_lgroup_t **group_p)
{
    return ucg_builtin_lgroup_create_ex(iface, group_id, member_count, my_index,
                                        combine, NULL, group_p);
}

void ucg_builtin_lgroup_destroy(ucg_builtin_lgroup_t *g)
{
    unsigned i;
    if (g == NULL) {
        return;
    }
    for (i = 0; i < UCG_BUILTIN_OPS_MAX_CONCURRENT; i++) {
        stash_t *m;
        while ((m = g->slots[i].msgs) != NULL) {
            g->slots[i].msgs = m->next;
            free(m);
        }
    }
    g->iface->groups[g->group_id % UNEXP_GROUPS] = NULL;
    rma_group_free(g);
    free(g);
}

unsigned ucg_builtin_lgroup_progress(ucg_builtin_lgroup_t *g)
{
    unsigned n = ucg_builtin_shm_progress(g->iface, am_handler, g->iface), i;
    /* resend queue (builtin.c:260-294, 329-337) */
    for (i = 0; i < UCG_BUILTIN_OPS_MAX_CONCURRENT; i++) {
        ucg_builtin_lcoll_t *c = g->slots[i].req;
        if (c && c->send_pending) {
            g->stats[3]++;
            if (c->rma) {
                rma_advance(c);
            } else {
                step_execute(c);
            }
            n++;
        }
    }
    return n;
}

void ucg_builtin_lgroup_stats(ucg_builtin_lgroup_t *g, uint64_t out[4])
{
    int i;
    for (i = 0; i < 4; i++) {
        out[i] = g ? g->stats[i] : 0;
    }
}

/* Fragmentation of one step's message (builtin_control.c:434,462-465) */
static ucs_status_t step_fragments(ucg_builtin_lcoll_t *c, op_step_t *s)
{
    size_t max_short   = ucg_builtin_shm_iface_max_short(c->g->iface);
    size_t max_payload = max_short - 8;
    if (c->length > max_payload) {
        s->frag_len = ucg_builtin_step_fragment_length(max_short, c->dt_len);
        if (s->frag_len == 0) {
            return UCS_ERR_UNSUPPORTED;
        }
        s->frags = ucg_builtin_step_fragments_total(c->length, s->frag_len, 1);
    } else {
        s->frag_len = 0;
        s->frags    = 1;
    }
    s->fragments_total = (uint64_t)s->recv_cnt * s->frags;
    return UCS_OK;
}

/* ---- plan construction (builtin/plan) ------------------------------------
 * The reference builds every tree for root 0 (builtin_tree.c:544-551) and a
 * non-zero root through ucg_builtin_topo_tree_set_root, which reads tree
 * parameters out of a plan phase (:590-592). Here a plan is built in a
 * virtual numbering in which the root is member 0: the root's host moves to
 * the front and the root to the front of its host, so hosts stay runs of
 * consecutive indices; v2r maps a virtual member back. */
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

/* The virtual numbering for `root`. Hosts are runs of ppn consecutive
 * members (the "by node" allocation builtin_tree.c:397-405 assumes); a layout
 * that is not, as seen from this member, is UCS_ERR_UNSUPPORTED. */
static ucs_status_t plan_ctx_init(ucg_builtin_lgroup_t *g, unsigned root, plan_ctx_t *pc)
{
    unsigned m, ppn = 0, H, hr, lr, r2v_my = 0;
    for (m = 0; m < g->size; m++) {
        ppn += g->distance[m] <= D_HOST;
    }
    if (ppn == 0 || g->size % ppn) {
        return UCS_ERR_UNSUPPORTED;
    }
    for (m = 0; m < g->size; m++) {
        if ((g->distance[m] <= D_HOST) != (m / ppn == g->my / ppn)) {
            return UCS_ERR_UNSUPPORTED;
        }
    }
    H  = g->size / ppn;
    hr = root / ppn;
    lr = root % ppn;
    pc->n           = g->size;
    pc->radix       = g->radix;
    pc->sock_thresh = g->sock_thresh;
    pc->factor      = g->factor;
    for (m = 0; m < g->size; m++) {
        unsigned vb = m / ppn, vi = m % ppn, li;
        li = (vb != 0) ? vi : (vi == 0) ? lr : (vi <= lr ? vi - 1 : vi);
        pc->v2r[m] = ((vb + hr) % H) * ppn + li;
        if (pc->v2r[m] == g->my) {
            r2v_my = m;
        }
    }
    pc->my = r2v_my;
    for (m = 0; m < g->size; m++) {
        uint8_t d = g->distance[pc->v2r[m]];
        /* with the root moved to the front of its host, sockets are no
         * longer runs of the virtual numbering: one intra-host level */
        pc->d[m] = (root != 0 && d == D_SOCKET) ? D_HOST : d;
    }
    return UCS_OK;
}

/* ucg_builtin_tree_add_intra, builtin_tree.c:262-380 (root 0): my parent is
 * the first member before me at the smallest distance; my children are the
 * members after me at a distance above the last one taken and within my
 * master phase - the first of each new distance moved to the front - and
 * the members at the distance of my first child. Below sock_thresh members
 * per host SOCKET counts as HOST (one level). */
static ucs_status_t tree_add_intra(const plan_ctx_t *pc, unsigned *ppn, unsigned *up,
                                   unsigned *up_cnt, unsigned *down, unsigned *down_cnt,
                                   unsigned *master_phase)
{
    unsigned m, up_distance = D_LAST, down_distance = D_SELF, first_distance = D_SELF;
    int single;
    *ppn = *up_cnt = *down_cnt = 0;
    *master_phase = D_NET;
    for (m = 0; m < pc->n; m++) {
        *ppn += pc->d[m] <= D_HOST;
    }
    single = *ppn < pc->sock_thresh;
    for (m = 0; m < pc->my; m++) {
        unsigned d = (single && pc->d[m] == D_SOCKET) ? D_HOST : pc->d[m];
        if (up_distance > d) {
            up_distance   = d;
            *master_phase = d - 1;
            up[0]         = m;
            *up_cnt       = 1;
        }
    }
    for (m = pc->my + 1; m < pc->n; m++) {
        unsigned d = (single && pc->d[m] == D_SOCKET) ? D_HOST : pc->d[m];
        if (d > down_distance && d <= *master_phase && d < D_NET) {
            down_distance  = d;
            first_distance = (first_distance == D_SELF) ? d : D_LAST;
            if (*down_cnt) {
                down[(*down_cnt)++] = down[0];
            } else {
                (*down_cnt)++;
            }
            down[0] = m;
        } else if (d == first_distance) {
            down[(*down_cnt)++] = m;
        }
        if (*down_cnt == TREE_MAX_RADIX) {
            return UCS_ERR_UNSUPPORTED;
        }
    }
    return UCS_OK;
}

/* The intra-host trees tree_add_intra cannot build: the host master takes
 * the first other socket's master as a child and no later one
 * (first_distance turns LAST, builtin_tree.c:336-351), so on a host of more
 * than two sockets (or with a CACHE level inside a socket) some masters send
 * to a parent that never expects them. UCS_ERR_UNSUPPORTED instead of a hang
 * (DESIGN.md 7). */
static ucs_status_t check_host_tree(const plan_ctx_t *pc)
{
    unsigned m, ppn = 0, sock = 0;
    int has_socket = 0;
    for (m = 0; m < pc->n; m++) {
        if (pc->d[m] == UCG_BUILTIN_DISTANCE_CACHE) {
            return UCS_ERR_UNSUPPORTED;
        }
        ppn        += pc->d[m] <= D_HOST;
        sock       += pc->d[m] <= D_SOCKET;
        has_socket |= pc->d[m] == D_SOCKET;
    }
    if (ppn >= pc->sock_thresh && has_socket && (ppn % sock || ppn / sock > 2)) {
        return UCS_ERR_UNSUPPORTED;
    }
    return UCS_OK;
}

/* ucg_builtin_tree_add_inter, builtin_tree.c:382-438: the hosts' masters
 * (every ppn-th member) form a tree of the given radix, root 0 */
static ucs_status_t tree_add_inter(const plan_ctx_t *pc, unsigned ppn, unsigned *up,
                                   unsigned *up_cnt, unsigned *down, unsigned *down_cnt)
{
    const unsigned long limit = pc->n, radix = pc->radix < 2 ? 2 : pc->radix;
    unsigned long inner_range = ppn, outer_range = (unsigned long)ppn * radix;
    unsigned long outer, inner, root;
    *up_cnt = *down_cnt = 0;
    do {
        for (outer = 0; outer < limit; outer += outer_range) {
            root = (outer_range < limit) ? outer : 0;
            for (inner = outer; inner < outer + outer_range && inner < limit;
                 inner += inner_range) {
                if (pc->my == inner) {
                    if (pc->my == root) {
                        continue;
                    }
                    up[(*up_cnt)++] = (unsigned)root;
                    if (*up_cnt == TREE_MAX_RADIX) {
                        return UCS_ERR_UNSUPPORTED;
                    }
                } else if (pc->my == root) {
                    down[(*down_cnt)++] = (unsigned)inner;
                    if (*down_cnt == TREE_MAX_RADIX) {
                        return UCS_ERR_UNSUPPORTED;
                    }
                }
            }
        }
        inner_range *= radix;
        outer_range *= radix;
    } while (outer_range < limit * radix);
    return UCS_OK;
}

/* one phase: who the step sends to and receives from, by method
 * (builtin_control.c:375-396 for the order, :960-972 for the aggregation) */
static ucs_status_t add_phase(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc,
                              op_method_t method, unsigned step_idx,
                              const unsigned *peers, unsigned npeers)
{
    op_step_t *s;
    unsigned i, first_send = 0, send_cnt = 0, recv_cnt = 0;
    if (c->nsteps == OPS_MAX_STEPS || npeers == 0 || npeers > PM || step_idx > 255) {
        return UCS_ERR_UNSUPPORTED;
    }
    s = &c->steps[c->nsteps++];
    memset(s, 0, sizeof(*s));
    s->method   = (uint8_t)method;
    s->step_idx = (uint8_t)step_idx;
    switch (method) {
    case M_SEND_TERMINAL:
    case M_SEND_TO_SM_ROOT:
        send_cnt = npeers;
        break;
    case M_REDUCE_TERMINAL:
        recv_cnt       = npeers;
        s->aggregation = AGG_REDUCE;
        break;
    case M_RECV_TERMINAL:
        recv_cnt       = npeers;
        s->aggregation = AGG_WRITE;
        break;
    case M_REDUCE_RECURSIVE:
        send_cnt = recv_cnt = npeers;
        s->aggregation = AGG_REDUCE;
        break;
    case M_REDUCE_WAYPOINT:      /* children first, the parent last */
        if (npeers < 2) {
            return UCS_ERR_UNSUPPORTED;
        }
        recv_cnt       = npeers - 1;
        first_send     = npeers - 1;
        send_cnt       = 1;
        s->aggregation = AGG_REDUCE;
        s->recv_first  = 1;
        break;
    case M_BCAST_WAYPOINT:       /* the parent first, then the children */
        if (npeers < 2) {
            return UCS_ERR_UNSUPPORTED;
        }
        recv_cnt       = 1;
        first_send     = 1;
        send_cnt       = npeers - 1;
        s->aggregation = AGG_WRITE;
        s->recv_first  = 1;
        break;
    }
    s->send_cnt = send_cnt;
    s->recv_cnt = recv_cnt;
    for (i = 0; i < send_cnt; i++) {
        s->send_peers[i] = pc->v2r[peers[first_send + i]];
    }
    for (i = 0; i < recv_cnt; i++) {
        s->recv_peers[i] = pc->v2r[peers[i]];
    }
    return UCS_OK;
}

/* ucg_builtin_tree_connect, builtin_tree.c:86-260, for the aggregating
 * collectives (AGGREGATE; BROADCAST for the fan-out of an allreduce): the
 * host fan-in at step_offset, the network fan-in at +1, the network fan-out
 * at +2 and the host fan-out at +3. A fan-in sends to the parent appended
 * after the children; a fan-out hears from the parent listed first. */
static ucs_status_t tree_connect(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc, int fanin,
                                 int fanout, unsigned step_offset, unsigned ppn,
                                 const unsigned *host_up, unsigned host_up_cnt,
                                 const unsigned *net_up, unsigned net_up_cnt,
                                 const unsigned *net_down, unsigned net_down_cnt,
                                 const unsigned *host_down, unsigned host_down_cnt)
{
    unsigned peers[2 * PM + 2], n, i;
    ucs_status_t st = UCS_OK;
    op_method_t method;
    if (fanin && host_up_cnt + host_down_cnt) {
        method = host_down_cnt ? (host_up_cnt ? M_REDUCE_WAYPOINT : M_REDUCE_TERMINAL) :
                 (ppn == 2) ? M_SEND_TERMINAL : M_SEND_TO_SM_ROOT;
        for (n = 0, i = 0; i < host_down_cnt; i++) peers[n++] = host_down[i];
        if (host_up_cnt) peers[n++] = host_up[0];
        st = add_phase(c, pc, method, step_offset, peers, n);
    }
    if (st == UCS_OK && fanin && net_up_cnt + net_down_cnt) {
        method = net_down_cnt ? (net_up_cnt ? M_REDUCE_WAYPOINT : M_REDUCE_TERMINAL) :
                 M_SEND_TERMINAL;
        for (n = 0, i = 0; i < net_down_cnt; i++) peers[n++] = net_down[i];
        if (net_up_cnt) peers[n++] = net_up[0];
        st = add_phase(c, pc, method, step_offset + 1, peers, n);
    }
    if (st == UCS_OK && fanout && net_up_cnt + net_down_cnt) {
        method = net_down_cnt ? (net_up_cnt ? M_BCAST_WAYPOINT : M_SEND_TERMINAL) :
                 M_RECV_TERMINAL;
        for (n = 0, i = 0; i < net_up_cnt; i++) peers[n++] = net_up[i];
        for (i = 0; i < net_down_cnt; i++) peers[n++] = net_down[i];
        st = add_phase(c, pc, method, step_offset + 2, peers, n);
    }
    if (st == UCS_OK && fanout && host_up_cnt + host_down_cnt) {
        method = host_down_cnt ? (host_up_cnt ? M_BCAST_WAYPOINT : M_SEND_TERMINAL) :
                 M_RECV_TERMINAL;
        for (n = 0, i = 0; i < host_up_cnt; i++) peers[n++] = host_up[i];
        for (i = 0; i < host_down_cnt; i++) peers[n++] = host_down[i];
        st = add_phase(c, pc, method, step_offset + 3, peers, n);
    }
    return st;
}

/* ucg_builtin_tree_create / _build, builtin_tree.c:441-561: the intra-host
 * tree, and for a host master of a multi-host group the inter-host tree (its
 * parent "of index 0" from the intra-host pass dropped, :488-497) */
static ucs_status_t plan_tree(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc, int fanout,
                              unsigned *ppn)
{
    unsigned host_up[PM], host_down[PM], net_up[TREE_MAX_RADIX], net_down[TREE_MAX_RADIX];
    unsigned hu, hd, nu = 0, nd = 0, mp;
    ucs_status_t st = check_host_tree(pc);
    if (st != UCS_OK || (st = tree_add_intra(pc, ppn, host_up, &hu, host_down, &hd,
                                             &mp)) != UCS_OK) {
        return st;
    }
    if (mp >= D_HOST && *ppn < pc->n) {
        hu = 0;
        if ((st = tree_add_inter(pc, *ppn, net_up, &nu, net_down, &nd)) != UCS_OK) {
            return st;
        }
    }
    c->plan = "tree";
    return tree_connect(c, pc, 1, fanout, 1, *ppn, host_up, hu, net_up, nu, net_down, nd,
                        host_down, hd);
}

/* ucg_builtin_recursive_create, builtin_recursive.c:20-228: recursive K-ing
 * (K = factor) over the hosts' masters - step k's peers are
 *   base + ((my - base + step_size * j) % (step_size * K)),  j = 1 .. K-1,
 *   base = my - my % (step_size * K), step_size = ppn * K^(k-1)
 * (:158-197) - wrapped in the intra-host fan-in and fan-out when hosts hold
 * several members. One host whose size is not a power of K runs the
 * intra-host tree alone (:78-82); several hosts whose number is not one are
 * UCS_ERR_UNSUPPORTED (:83-87). */
static ucs_status_t plan_recursive(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc,
                                   unsigned *ppn_out)
{
    unsigned host_up[PM], host_down[PM], peers[PM];
    unsigned ppn, hu, hd, mp, steps = 0, k, j, idx;
    unsigned long proc_count, step_size = 1;
    ucs_status_t st = tree_add_intra(pc, &ppn, host_up, &hu, host_down, &hd, &mp);
    if (st != UCS_OK) {
        return st;
    }
    *ppn_out = ppn;
    /* a host's master drops its parent from the intra-host pass (a member
     * of another host). The reference tests master_phase == HOST (:55),
     * which no NET parent produces; >= HOST is the intent */
    if (mp >= D_HOST) {
        hu = 0;
    }
    if (pc->factor < 2) {
        return UCS_ERR_INVALID_PARAM;
    }
    proc_count = (pc->n == ppn) ? ppn : pc->n / ppn + (pc->n % ppn > 0);
    while (step_size < proc_count) {
        step_size *= pc->factor;
        steps++;
    }
    if (step_size != proc_count) {
        if (pc->n != ppn) {
            return UCS_ERR_UNSUPPORTED;
        }
        steps = 0;               /* one host: the intra-host tree */
    }
    if (pc->n == ppn && steps) {
        hu = hd = 0;             /* one host, recursive among all members */
        ppn = 1;
    } else if ((st = check_host_tree(pc)) != UCS_OK) {
        return st;
    }
    if (steps == 0) {
        c->plan = "tree";
    } else if (hu || hd) {
        c->plan = pc->factor == 2 ? "host fan-in, recursive doubling over host masters, fan-out" :
                                    "host fan-in, recursive K-ing over host masters, fan-out";
    } else {
        c->plan = pc->factor == 2 ? "recursive doubling" : "recursive K-ing";
    }
    if ((hu || hd) &&
        (st = tree_connect(c, pc, 1, 0, 1, ppn, host_up, hu, NULL, 0, NULL, 0,
                           host_down, hd)) != UCS_OK) {
        return st;
    }
    if (!hu) {
        idx = c->nsteps + 1;
        step_size = ppn;
        for (k = 0; k < steps; k++, step_size *= pc->factor) {
            unsigned long base = pc->my - pc->my % (step_size * pc->factor);
            for (j = 1; j < pc->factor; j++) {
                peers[j - 1] = (unsigned)(base + ((pc->my - base + step_size * j) %
                                                  (step_size * pc->factor)));
            }
            if ((st = add_phase(c, pc, M_REDUCE_RECURSIVE, idx + k, peers,
                                pc->factor - 1)) != UCS_OK) {
                return st;
            }
        }
    }
    if (hu || hd) {
        st = tree_connect(c, pc, 0, 1, steps + 1, ppn, host_up, hu, NULL, 0, NULL, 0,
                          host_down, hd);
    }
    return st;
}

/* what every step of the member's plan sends and how much it receives:
 * the send buffer is recv.buffer once anything was received into it
 * (builtin_control.c:673-683; a waypoint sends what it received), the
 * accumulator is seeded (ucg_builtin_init_reduce) when the member reduces,
 * and the SM-root children of a one-level host fan-in may pack into one
 * incast cell at their master (builtin_control.c:535-537) */
/* The reference forwards every fragmented waypoint fragment by fragment
 * (builtin_control.c:831-834). On the shared-memory transport of this engine
 * that is slower (early fragments land in the parent's stash
 * while it still fans in), so it is off unless UCX_BUILTIN_PIPELINE=y. */
static int pipeline_enabled(void)
{
    const char *e = getenv("UCX_BUILTIN_PIPELINE");
    return e && (e[0] == 'y' || e[0] == 'Y' || e[0] == '1');
}

static ucs_status_t plan_finish(ucg_builtin_lcoll_t *c, unsigned ppn)
{
    ucg_builtin_lgroup_t *g = c->g;
    int received = 0;
    unsigned k;
    c->init_reduce = 0;
    c->pipe_cap    = 0;
    for (k = 0; k < c->nsteps; k++) {
        op_step_t *s = &c->steps[k];
        s->send_recv_buffer = received || s->recv_first;
        if (s->recv_cnt) {
            received = 1;
        }
        if (s->aggregation == AGG_REDUCE) {
            c->init_reduce = 1;
        }
        if (step_fragments(c, s) != UCS_OK) {
            return UCS_ERR_UNSUPPORTED;
        }
        s->pipelined = s->recv_first && s->frag_len && pipeline_enabled();
        if (s->pipelined && s->frags > c->pipe_cap) {
            c->pipe_cap = s->frags;
        }
        if (g->incast && s->step_idx == 1 && ppn > 2 && ppn < g->sock_thresh) {
            if (s->method == M_REDUCE_TERMINAL) {
                s->incast          = 1;
                s->fragments_total = s->frags;
            } else if (s->method == M_SEND_TO_SM_ROOT) {
                s->incast          = 1;
                s->incast_expected = ppn - 1;
                s->packer = ucg_builtin_combine_atomic_sum_length(g->cmb, c->op, c->dtype)
                            ? PACK_ATOMIC : PACK_REDUCING;
            }
        }
    }
    if (c->pipe_cap) {
        /* one count per fragment (the reference allocates sizeof(ep_cnt)
         * bytes for frags_per_ep counts, builtin_control.c:738-739 against
         * builtin_data.c:433) */
        c->frag_left = malloc(c->pipe_cap * sizeof(*c->frag_left));
        c->frag_fifo = malloc(c->pipe_cap * sizeof(*c->frag_fifo));
        if (c->frag_left == NULL || c->frag_fifo == NULL) {
            return UCS_ERR_NO_MEMORY;
        }
    }
    return UCS_OK;
}

/* ------------------------------------------------------------------------ */
/* device-resident buffers: remote-key steps                                */
/* ------------------------------------------------------------------------ */
/* An op whose buffers are GPU memory runs the same plan, but no data crosses
 * the AM transport: every member keeps its data in a device buffer of its
 * own, exposed to the peers that read it through a HIP IPC handle - the
 * packed remote key of the reference's rkey-exchange step
 * (ucg_builtin_step_create_rkey_bcast, builtin_control.c:1014-1076), sent
 * once per op since the buffers outlive every start. A step's send becomes
 * READY (my buffer b holds what you would receive) and its receive becomes one
 * kernel reading the senders' buffers over xGMI (SEND_GET_ZCOPY,
 * builtin_data.c:326-340), after which the reader answers DONE so the sender
 * may write that buffer again. Two buffers per member alternate, so a member
 * never waits for readers of the data it is combining into: step k reads
 * dbuf[cur] and writes dbuf[!cur] unless nobody reads dbuf[cur]. The
 * association is the host path's: the accumulator first, then the peers in
 * the order their READYs arrived (builtin_comp_step.inl:213-221). */
#define RMA_DONE 0x40   /* payload {from, buf}: done reading your dbuf[buf] */
#define RMA_RKEY 0x80   /* payload {from, buf, handle}: the key of my dbuf[buf] */
#define RMA_MIN_SHORT (8 + 8 + UCG_BUILTIN_DEV_IPC_HANDLE_BYTES)

struct rma_msg {
    unsigned peer;
    uint64_t header;
    uint32_t length;
    uint8_t  payload[8 + UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
};

#define RMA_DEV 1       /* device buffers: HIP IPC keys, kernels */
#define RMA_SHM 2       /* host buffers: POSIX shared memory keys, reduce_cb_f */

struct rma_pool {
    void    *ptr;
    size_t   bytes;
    int      kind;
    int      busy;
    uint8_t  key[UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
};

struct rma_imp {
    unsigned peer;
    int      kind;
    uint8_t  key[UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
    void    *ptr;
};

/* Host buffers behind the same steps: the op's buffers are POSIX shared
 * memory segments and a key names one (the reference's remote-key step
 * serves "both shared memory and network", builtin_control.c:712-719). A
 * zero-copy step for large host messages, as the reference switches to
 * zcopy above its 100000-byte threshold (builtin_control.c:474). */
typedef struct {
    uint32_t magic;
    uint32_t pad;
    uint64_t bytes;
    char     name[64];
} shm_key_t;

_Static_assert(sizeof(shm_key_t) <= UCG_BUILTIN_DEV_IPC_HANDLE_BYTES, "shm key size");
#define SHM_KEY_MAGIC 0x4d485358u

static void *shm_seg_alloc(size_t bytes, void *key)
{
    static _Atomic unsigned seq;
    shm_key_t k;
    void *p;
    int fd;
    memset(&k, 0, sizeof(k));
    k.magic = SHM_KEY_MAGIC;
    k.bytes = bytes;
    snprintf(k.name, sizeof(k.name), "/xucg_rma_%d_%u", (int)getpid(),
             atomic_fetch_add(&seq, 1));
    fd = shm_open(k.name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) {
        return NULL;
    }
    if (ftruncate(fd, (off_t)bytes) != 0) {
        close(fd);
        shm_unlink(k.name);
        return NULL;
    }
    p = mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        shm_unlink(k.name);
        return NULL;
    }
    memset(key, 0, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
    memcpy(key, &k, sizeof(k));
    return p;
}

static ucs_status_t shm_seg_import(const void *key, void **ptr)
{
    shm_key_t k;
    void *p;
    int fd;
    memcpy(&k, key, sizeof(k));
    if (k.magic != SHM_KEY_MAGIC || memchr(k.name, 0, sizeof(k.name)) == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    fd = shm_open(k.name, O_RDWR, 0);
    if (fd < 0) {
        return UCS_ERR_IO_ERROR;
    }
    p = mmap(NULL, k.bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        return UCS_ERR_NO_MEMORY;
    }
    *ptr = p;
    return UCS_OK;
}

static size_t shm_key_bytes(const void *key)
{
    shm_key_t k;
    memcpy(&k, key, sizeof(k));
    return (size_t)k.bytes;
}

/* a free registered buffer of exactly `bytes`, or a new one */
static int rma_pool_get(ucg_builtin_lgroup_t *g, size_t bytes, int kind)
{
    struct rma_pool *p;
    unsigned i;
    for (i = 0; i < g->npool; i++) {
        if (!g->pool[i].busy && g->pool[i].bytes == bytes && g->pool[i].kind == kind) {
            g->pool[i].busy = 1;
            return (int)i;
        }
    }
    p = realloc(g->pool, (g->npool + 1) * sizeof(*p));
    if (p == NULL) {
        return -1;
    }
    g->pool = p;
    p = &g->pool[g->npool];
    p->bytes = bytes;
    p->kind  = kind;
    p->busy  = 1;
    if (kind == RMA_SHM) {
        p->ptr = shm_seg_alloc(bytes, p->key);
        return p->ptr ? (int)g->npool++ : -1;
    }
    p->ptr = ucg_builtin_combine_dev_alloc(g->cmb, bytes);
    if (p->ptr == NULL) {
        return -1;
    }
    if (ucg_builtin_combine_dev_export(g->cmb, p->ptr, p->key) != UCS_OK) {
        ucg_builtin_combine_dev_free(g->cmb, p->ptr);
        return -1;
    }
    return (int)g->npool++;
}

/* a peer's buffer by its key: mapped once per group */
static ucs_status_t rma_import(ucg_builtin_lgroup_t *g, unsigned peer, int kind,
                               const void *key, void **ptr)
{
    struct rma_imp *m;
    unsigned i;
    ucs_status_t st;
    for (i = 0; i < g->nimp; i++) {
        if (g->imp[i].peer == peer && g->imp[i].kind == kind &&
            memcmp(g->imp[i].key, key, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES) == 0) {
            *ptr = g->imp[i].ptr;
            return UCS_OK;
        }
    }
    m = realloc(g->imp, (g->nimp + 1) * sizeof(*m));
    if (m == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    g->imp = m;
    st = (kind == RMA_SHM) ? shm_seg_import(key, ptr) :
                             ucg_builtin_combine_dev_import(g->cmb, key, ptr);
    if (st != UCS_OK) {
        return st;
    }
    m = &g->imp[g->nimp++];
    m->peer = peer;
    m->kind = kind;
    memcpy(m->key, key, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
    m->ptr = *ptr;
    return UCS_OK;
}

static void rma_group_free(ucg_builtin_lgroup_t *g)
{
    unsigned i;
    for (i = 0; i < g->nimp; i++) {
        if (g->imp[i].kind == RMA_SHM) {
            munmap(g->imp[i].ptr, shm_key_bytes(g->imp[i].key));
        } else {
            ucg_builtin_combine_dev_release(g->cmb, g->imp[i].ptr);
        }
    }
    for (i = 0; i < g->npool; i++) {
        if (g->pool[i].kind == RMA_SHM) {
            shm_key_t k;
            memcpy(&k, g->pool[i].key, sizeof(k));
            munmap(g->pool[i].ptr, g->pool[i].bytes);
            shm_unlink(k.name);
        } else {
            ucg_builtin_combine_dev_free(g->cmb, g->pool[i].ptr);
        }
    }
    free(g->imp);
    free(g->pool);
}

/* UCX_BUILTIN_SHM_ZCOPY_THRESH: host messages of at least this many bytes
 * take the shared-memory remote-key steps (0 or unset = never; this build's
 * knob - the reference hard-codes 100000, builtin_control.c:474) */
static size_t shm_zcopy_thresh(void)
{
    const char *e = getenv("UCX_BUILTIN_SHM_ZCOPY_THRESH");
    return (e && *e) ? (size_t)strtoull(e, NULL, 0) : 0;
}

/* the op's buffers decide: device memory (both, or the one given) ->
 * RMA_DEV, large host messages with the knob -> RMA_SHM, other host
 * memory -> 0, one of each -> -1 */
static int rma_kind(ucg_builtin_lgroup_t *g, const void *sbuf, const void *rbuf,
                    size_t length)
{
    int sk, rk;
    const size_t thresh = shm_zcopy_thresh();
    if (ucg_builtin_combine_has_device(g->cmb)) {
        sk = sbuf ? ucg_builtin_dev_mem_kind(sbuf) : -1;
        rk = rbuf ? ucg_builtin_dev_mem_kind(rbuf) : -1;
        if (sk == UCG_DEV_MEM_DEVICE || rk == UCG_DEV_MEM_DEVICE) {
            return (sbuf && sk != UCG_DEV_MEM_DEVICE) ||
                   (rbuf && rk != UCG_DEV_MEM_DEVICE) ? -1 : RMA_DEV;
        }
    }
    return (thresh && length >= thresh) ? RMA_SHM : 0;
}

/* the receive's combine: dst = srcs[n-1] (op) (... (srcs[1] (op) srcs[0])) */
static ucs_status_t rma_fold(ucg_builtin_lcoll_t *c, void *dst, const void *const *srcs,
                             unsigned n)
{
    unsigned m;
    ucs_status_t st = UCS_OK;
    if (c->rma == RMA_DEV) {
        return ucg_builtin_combine_dev_fold(c->g->cmb, c->op, c->dtype, dst, srcs, n,
                                            (size_t)c->count);
    }
    if (dst != srcs[0]) {
        memcpy(dst, srcs[0], c->length);
    }
    for (m = 1; m < n && st == UCS_OK; m++) {
        st = ucg_builtin_combine_reduce(c->g->cmb, c->op, (void*)srcs[m], dst, c->count,
                                        c->dtype);
    }
    return st;
}

static ucs_status_t rma_copy(ucg_builtin_lcoll_t *c, void *dst, const void *src)
{
    if (c->rma == RMA_DEV) {
        return ucg_builtin_combine_dev_copy(c->g->cmb, dst, src, c->length);
    }
    if (dst != src) {
        memcpy(dst, src, c->length);
    }
    return UCS_OK;
}

static void rma_post(ucg_builtin_lcoll_t *c, unsigned peer, uint8_t kind,
                     unsigned buf, const void *extra, size_t extra_len)
{
    struct rma_msg *m;
    ops_header_t h;
    uint32_t w[2] = {c->g->my, buf};
    if (c->out_tail == c->out_cap) {
        unsigned cap = c->out_cap ? 2 * c->out_cap : 64;
        struct rma_msg *o = realloc(c->outbox, cap * sizeof(*o));
        if (o == NULL) {
            finish(c, UCS_ERR_NO_MEMORY);
            return;
        }
        c->outbox  = o;
        c->out_cap = cap;
    }
    m = &c->outbox[c->out_tail++];
    h.header   = 0;
    h.group_id = c->g->group_id;
    h.coll_id  = c->coll_id;
    h.step_idx = kind;
    m->peer    = peer;
    m->header  = h.header;
    m->length  = (uint32_t)(8 + extra_len);
    memcpy(m->payload, w, 8);
    if (extra_len) {
        memcpy(m->payload + 8, extra, extra_len);
    }
}

/* in order; resumed from lgroup_progress after UCS_ERR_NO_RESOURCE */
static void rma_flush(ucg_builtin_lcoll_t *c)
{
    while (!c->done && c->out_head < c->out_tail) {
        struct rma_msg *m = &c->outbox[c->out_head];
        ucs_status_t st = ucg_builtin_shm_am_short(c->g->iface, m->peer, m->header,
                                                   m->payload, m->length);
        if (st == UCS_ERR_NO_RESOURCE) {
            c->send_pending = 1;
            return;
        }
        if (st != UCS_OK) {
            finish(c, st);
            return;
        }
        c->g->stats[0]++;
        c->out_head++;
    }
    c->out_head = c->out_tail = 0;
    c->send_pending = 0;
}

/* the send half of a step: READY to every reader, who now holds one more
 * reference to the buffer */
static void rma_expose(ucg_builtin_lcoll_t *c, const op_step_t *s)
{
    unsigned e;
    for (e = 0; e < s->send_cnt; e++) {
        rma_post(c, s->send_peers[e], s->step_idx, c->cur_buf, NULL, 0);
    }
    c->readers[c->cur_buf] += s->send_cnt;
}

/* the receive half: once every sender's READY is in and the target buffer
 * has no readers left, one kernel; then DONE to every sender. 0 = wait. */
static int rma_receive(ucg_builtin_lcoll_t *c, const op_step_t *s)
{
    const unsigned k = c->cur;
    const void *srcs[UCG_BUILTIN_OPS_MAX_MEMBERS + 1];
    /* the last receive with nothing exposed after it writes the result
     * straight into recv.buffer (no final copy) */
    const int direct = c->rbuf_user && k + 1 == c->nsteps &&
                       !(s->recv_first && s->send_cnt);
    unsigned out, i;
    void *dst;
    ucs_status_t st;

    if (c->rdy_cnt[k] < s->recv_cnt) {
        return 0;
    }
    out = c->readers[c->cur_buf] ? !c->cur_buf : c->cur_buf;
    if (!direct && c->readers[out]) {
        return 0;
    }
    dst = direct ? (void*)c->rbuf_user : c->dbuf[out];
    for (i = 0; i < s->recv_cnt; i++) {
        srcs[1 + i] = c->peer_buf[c->rdy_peer[k][i]][c->rdy_buf[k][i]];
        if (srcs[1 + i] == NULL) {
            finish(c, UCS_ERR_IO_ERROR);      /* a READY without a key */
            return 0;
        }
    }
    if (s->aggregation == AGG_REDUCE) {
        srcs[0] = c->dbuf[c->cur_buf];
        st = rma_fold(c, dst, srcs, 1 + s->recv_cnt);
    } else {
        st = (s->recv_cnt == 1) ? rma_copy(c, dst, srcs[1]) : UCS_ERR_IO_ERROR;
    }
    if (st != UCS_OK) {
        finish(c, st);
        return 0;
    }
    for (i = 0; i < s->recv_cnt; i++) {
        rma_post(c, c->rdy_peer[k][i], RMA_DONE, c->rdy_buf[k][i], NULL, 0);
    }
    if (direct) {
        c->rma_final = 1;
    } else {
        c->cur_buf = out;
    }
    return 1;
}

/* as far as the messages in allow; the op completes once the result is in
 * recv.buffer and nobody reads this member's buffers any more */
static void rma_advance(ucg_builtin_lcoll_t *c)
{
    if (c->rma_busy) {
        c->rma_again = 1;
        return;
    }
    c->rma_busy = 1;
    do {
        c->rma_again = 0;
        rma_flush(c);
        while (!c->done && c->cur < c->nsteps) {
            const op_step_t *s = &c->steps[c->cur];
            if (!s->recv_first && !c->rma_sent) {
                rma_expose(c, s);
                c->rma_sent = 1;
            }
            if (s->recv_cnt && !c->rma_recvd) {
                if (!rma_receive(c, s)) {
                    break;
                }
                c->rma_recvd = 1;
            }
            if (s->recv_first && !c->rma_sent) {
                rma_expose(c, s);
                c->rma_sent = 1;
            }
            c->cur++;
            c->rma_sent = c->rma_recvd = 0;
        }
        if (!c->done && c->cur == c->nsteps && !c->rma_final) {
            ucs_status_t st = c->rbuf_user ?
                rma_copy(c, c->rbuf_user, c->dbuf[c->cur_buf]) : UCS_OK;
            if (st != UCS_OK) {
                finish(c, st);
            }
            c->rma_final = 1;
        }
        rma_flush(c);
        if (!c->done && c->rma_final && c->out_tail == 0 &&
            c->readers[0] == 0 && c->readers[1] == 0) {
            finish(c, UCS_OK);
        }
    } while (c->rma_again && !c->done);
    c->rma_busy = 0;
}

/* a control message of this op (am_handler, or the stash at start) */
static void rma_msg(ucg_builtin_lcoll_t *c, ops_header_t h, const void *data,
                    size_t length)
{
    uint32_t w[2];
    unsigned k;
    if (c->done) {
        return;
    }
    if (length < 8) {
        finish(c, UCS_ERR_IO_ERROR);
        return;
    }
    memcpy(w, data, 8);
    if (w[0] >= c->g->size || w[0] == c->g->my || w[1] > 1) {
        finish(c, UCS_ERR_IO_ERROR);   /* e.g. a member that took the host path */
        return;
    }
    if (h.step_idx == RMA_RKEY) {
        void *p = NULL;
        ucs_status_t st;
        if (length != 8 + UCG_BUILTIN_DEV_IPC_HANDLE_BYTES || c->peer_buf[w[0]][w[1]]) {
            finish(c, UCS_ERR_IO_ERROR);
            return;
        }
        st = rma_import(c->g, w[0], c->rma, (const char*)data + 8, &p);
        if (st != UCS_OK) {
            finish(c, st);
            return;
        }
        c->peer_buf[w[0]][w[1]] = p;
        return;                        /* nothing waits on a key alone */
    }
    if (h.step_idx == RMA_DONE) {
        if (c->readers[w[1]] == 0) {
            finish(c, UCS_ERR_IO_ERROR);
            return;
        }
        c->readers[w[1]]--;
    } else {
        for (k = 0; k < c->nsteps && c->steps[k].step_idx != h.step_idx; k++) {
        }
        if (k == c->nsteps || c->rdy_cnt[k] == c->steps[k].recv_cnt) {
            finish(c, UCS_ERR_IO_ERROR);
            return;
        }
        c->rdy_peer[k][c->rdy_cnt[k]] = (uint8_t)w[0];
        c->rdy_buf[k][c->rdy_cnt[k]]  = (uint8_t)w[1];
        c->rdy_cnt[k]++;
    }
    rma_advance(c);
}

/* at create: the op's own buffers and their keys */
static ucs_status_t rma_setup(ucg_builtin_lcoll_t *c, void *rbuf_user)
{
    ucg_dev_op_t o;
    ucg_dev_dtype_t d;
    unsigned i;
    if (ucg_builtin_shm_iface_max_short(c->g->iface) < RMA_MIN_SHORT ||
        (c->rma == RMA_DEV &&
         !ucg_builtin_combine_classify(c->g->cmb, c->op, c->dtype, &o, &d))) {
        return UCS_ERR_UNSUPPORTED;
    }
    c->rbuf_user = rbuf_user;
    for (i = 0; i < 2; i++) {
        int k = rma_pool_get(c->g, c->length ? c->length : 1, c->rma);
        if (k < 0) {
            return UCS_ERR_NO_MEMORY;
        }
        c->pool_idx[i] = k;
        c->dbuf[i]     = c->g->pool[k].ptr;
        memcpy(c->key[i], c->g->pool[k].key, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
    }
    return UCS_OK;
}

static ucs_status_t rma_start(ucg_builtin_lcoll_t *c, op_slot_t *slot)
{
    ucs_status_t st;
    unsigned k, e;
    stash_t **pp;

    c->cur       = 0;
    c->cur_buf   = 0;
    c->rma_sent  = c->rma_recvd = c->rma_final = 0;
    c->readers[0] = c->readers[1] = 0;
    c->out_head  = c->out_tail = 0;
    c->send_pending = 0;
    memset(c->rdy_cnt, 0, sizeof(c->rdy_cnt));
    if (c->length == 0) {
        c->done   = 1;
        c->status = UCS_OK;
        return UCS_OK;
    }
    /* ucg_builtin_init_reduce (builtin_control.c:43-47): this member's data
     * into its first buffer - every member, since every member exposes it */
    st = rma_copy(c, c->dbuf[0], c->sbuf ? c->sbuf : c->rbuf);
    if (st != UCS_OK) {
        c->done   = 1;
        c->status = st;
        return st;
    }
    c->done   = 0;
    c->status = UCS_INPROGRESS;
    c->active = 1;
    slot->req = c;
    c->rma_busy = 1;                  /* post and drain before advancing */
    if (!c->keys_sent) {
        /* the keys go to every member that reads from this one */
        uint8_t sent[UCG_BUILTIN_OPS_MAX_MEMBERS] = {0};
        for (k = 0; k < c->nsteps; k++) {
            for (e = 0; e < c->steps[k].send_cnt; e++) {
                unsigned p = c->steps[k].send_peers[e];
                if (!sent[p]) {
                    sent[p] = 1;
                    rma_post(c, p, RMA_RKEY, 0, c->key[0], UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
                    rma_post(c, p, RMA_RKEY, 1, c->key[1], UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
                }
            }
        }
        c->keys_sent = 1;
    }
    /* what arrived before this start (ucg_builtin_step_check_pending) */
    pp = &slot->msgs;
    while (*pp && !c->done) {
        stash_t *m = *pp;
        ops_header_t h;
        h.header = m->header;
        if (h.coll_id != c->coll_id) {
            pp = &m->next;
            continue;
        }
        *pp = m->next;
        if (m->next == NULL) {
            slot->msgs_tail = pp;
        }
        rma_msg(c, h, m->data, m->length);
        free(m);
    }
    c->rma_busy = 0;
    rma_advance(c);
    return c->done ? c->status : UCS_INPROGRESS;
}

/* the op's buffers go back to the group's pool; peers' mappings stay */
static void rma_free(ucg_builtin_lcoll_t *c)
{
    unsigned i;
    for (i = 0; i < 2; i++) {
        if (c->pool_idx[i] >= 0) {
            c->g->pool[c->pool_idx[i]].busy = 0;
        }
    }
    free(c->outbox);
}

static void lcoll_free(ucg_builtin_lcoll_t *c)
{
    if (c) {
        if (c->rma) {
            rma_free(c);
        }
        free(c->scratch);
        free(c->frag_left);
        free(c->frag_fifo);
    }
    free(c);
}

static ucs_status_t lcoll_new(ucg_builtin_lgroup_t *g, const void *sbuf,
                              void *rbuf, int count, void *dtype, void *op,
                              ucg_builtin_lcoll_t **coll_p)
{
    ucg_builtin_lcoll_t *c;
    size_t dt_len;
    int rma;

    if (g == NULL || coll_p == NULL || count < 0 || (count && sbuf == NULL)) {
        return UCS_ERR_INVALID_PARAM;
    }
    dt_len = ucg_builtin_combine_dtype_length(g->cmb, dtype);
    if (dt_len == 0) {
        return UCS_ERR_INVALID_PARAM;
    }
    rma = count ? rma_kind(g, sbuf, rbuf, (size_t)count * dt_len) : 0;
    if (rma < 0) {
        return UCS_ERR_UNSUPPORTED;   /* one buffer on the host, one on the GPU */
    }
    if (!rma && (size_t)count * dt_len * g->size > 0xffffffffull) {
        return UCS_ERR_UNSUPPORTED;   /* 32-bit remote_offset, SURVEY 7 (ix) */
    }
    c = calloc(1, sizeof(*c));
    if (c == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    c->g      = g;
    c->sbuf   = sbuf;
    c->rbuf   = rbuf;
    c->count  = count;
    c->dtype  = dtype;
    c->op     = op;
    c->dt_len = dt_len;
    c->length = (size_t)count * dt_len;
    c->rma    = rma;              /* buffers set up once the plan is known */
    c->pool_idx[0] = c->pool_idx[1] = -1;
    c->done   = 1;
    c->status = UCS_OK;
    *coll_p   = c;
    return UCS_OK;
}

/* UCX_BUILTIN_ALLREDUCE_PLAN=auto|tree|recursive (this build's knob; the
 * reference always takes ucg_builtin_choose_topology's choice) */
static int allreduce_use_tree(unsigned size)
{
    const char *p = getenv("UCX_BUILTIN_ALLREDUCE_PLAN");
    if (p && strcmp(p, "tree") == 0) {
        return 1;
    }
    if (p && strcmp(p, "recursive") == 0) {
        return 0;
    }
    return (size & (size - 1)) != 0;   /* builtin.c:112-121 */
}

ucs_status_t ucg_builtin_lcoll_allreduce(ucg_builtin_lgroup_t *g, const void *sbuf,
                                         void *rbuf, int count, void *dtype,
                                         void *op, ucg_builtin_lcoll_t **coll_p)
{
    ucg_builtin_lcoll_t *c;
    plan_ctx_t pc;
    unsigned ppn = 1;
    ucs_status_t st;

    if (rbuf == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    st = lcoll_new(g, sbuf, rbuf, count, dtype, op, &c);
    if (st != UCS_OK) {
        return st;
    }
    c->kind = 0;
    if (g->size == 1) {
        c->plan        = "none";
        c->init_reduce = 1;
        st = UCS_OK;
    } else if ((st = ucg_builtin_combine_check_reduction(g->cmb, op)) == UCS_OK &&
               (st = plan_ctx_init(g, 0, &pc)) == UCS_OK) {
        /* the reduction checks of builtin_control.c:872-888 are made by every
         * member, not only by those with a reducing step: a leaf that went
         * ahead would wait for a fan-out nobody sends */
        st = allreduce_use_tree(g->size) ? plan_tree(c, &pc, 1, &ppn) :
                                           plan_recursive(c, &pc, &ppn);
        if (st == UCS_OK) {
            st = plan_finish(c, ppn);
        }
    }
    if (st == UCS_OK && c->rma) {
        st = rma_setup(c, rbuf);
    }
    if (st != UCS_OK) {
        lcoll_free(c);
        return st;
    }
    *coll_p = c;
    return UCS_OK;
}

ucs_status_t ucg_builtin_lcoll_reduce(ucg_builtin_lgroup_t *g, const void *sbuf,
                                      void *rbuf, int count, void *dtype,
                                      void *op, unsigned root,
                                      ucg_builtin_lcoll_t **coll_p)
{
    ucg_builtin_lcoll_t *c;
    plan_ctx_t pc;
    unsigned ppn = 1, k;
    ucs_status_t st;

    if (g == NULL || root >= g->size || (g->my == root && rbuf == NULL)) {
        return UCS_ERR_INVALID_PARAM;
    }
    st = lcoll_new(g, sbuf, rbuf, count, dtype, op, &c);
    if (st != UCS_OK) {
        return st;
    }
    c->kind = 1;
    c->root = root;
    if (g->size == 1) {
        c->plan        = "none";
        c->init_reduce = 1;
    } else if ((st = ucg_builtin_combine_check_reduction(g->cmb, op)) != UCS_OK ||
               (st = plan_ctx_init(g, root, &pc)) != UCS_OK ||
               (st = plan_tree(c, &pc, 0, &ppn)) != UCS_OK ||
               (st = plan_finish(c, ppn)) != UCS_OK) {
        lcoll_free(c);
        return st;
    }
    if (c->rma) {
        if ((st = rma_setup(c, g->my == root ? rbuf : NULL)) != UCS_OK) {
            lcoll_free(c);
            return st;
        }
        *coll_p = c;
        return UCS_OK;
    }
    /* a member other than the root that combines on the way (a host master,
     * a waypoint) accumulates in a buffer of the op's own: MPI leaves recvbuf
     * undefined off the root */
    for (k = 0; k < c->nsteps && g->my != root; k++) {
        if (c->steps[k].aggregation != AGG_NOP) {
            c->scratch = malloc(c->length ? c->length : 1);
            if (c->scratch == NULL) {
                lcoll_free(c);
                return UCS_ERR_NO_MEMORY;
            }
            c->rbuf = c->scratch;
            break;
        }
    }
    *coll_p = c;
    return UCS_OK;
}

ucs_status_t ucg_builtin_lcoll_start(ucg_builtin_lcoll_t *c)
{
    ucg_builtin_lgroup_t *g;
    op_slot_t *slot;

    if (c == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (c->active) {
        return UCS_ERR_BUSY;
    }
    g = c->g;
    c->coll_id = g->next_coll_id;
    slot = &g->slots[c->coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT];
    if (slot->req != NULL) {
        return UCS_ERR_BUSY;    /* more than 16 ops outstanding */
    }
    g->next_coll_id++;          /* ucg_collective_trigger, base/ucg_group.c:485 */
    if (c->rma) {
        return rma_start(c, slot);
    }
    /* ucg_builtin_init_reduce: recv <- send (in place: nothing to copy);
     * tree leaves have no init (builtin_control.c:755-767) */
    if (c->init_reduce && c->rbuf != c->sbuf && c->length) {
        memcpy(c->rbuf, c->sbuf, c->length);
    }
    c->done         = 0;
    c->status       = UCS_INPROGRESS;
    c->cur          = 0;
    c->step_open    = 0;
    c->step_started = 0;
    c->send_pending = 0;
    if (c->nsteps == 0 || c->length == 0) {
        c->done   = 1;
        c->status = UCS_OK;
        return UCS_OK;
    }
    c->active = 1;
    slot->req = c;
    step_execute(c);
    return c->done ? c->status : UCS_INPROGRESS;
}

int ucg_builtin_lcoll_test(ucg_builtin_lcoll_t *c, ucs_status_t *status)
{
    if (c->done && status) {
        *status = c->status;
    }
    return c->done;
}

ucs_status_t ucg_builtin_lcoll_wait(ucg_builtin_lcoll_t *c)
{
    static double lim = -1.0;
    static long spin = -1;
    unsigned idle = 0;
    double t0 = now_s();
    if (lim < 0.0) {
        const char *e = getenv("UCX_BUILTIN_WAIT_SPIN");
        lim  = wait_timeout_s();
        spin = e ? atol(e) : 4096;
    }
    while (!c->done) {
        if (ucg_builtin_lgroup_progress(c->g) != 0) {
            idle = 0;
            continue;
        }
        /* a peer's message is usually a few hundred ns away: spin first,
         * give the core away only when the wait gets long */
        if (++idle < (unsigned long)spin) {
            __builtin_ia32_pause();
            continue;
        }
        if (now_s() - t0 > lim) {
            finish(c, UCS_ERR_TIMED_OUT);
            break;
        }
        sched_yield();
    }
    return c->status;
}

void ucg_builtin_lcoll_destroy(ucg_builtin_lcoll_t *c)
{
    if (c && c->active) {
        finish(c, UCS_ERR_CANCELED);
    }
    lcoll_free(c);
}

size_t ucg_builtin_lcoll_describe(ucg_builtin_lcoll_t *c, char *buf, size_t max)
{
    size_t w = 0;
    unsigned k;
    if (c == NULL || buf == NULL || max == 0) {
        return 0;
    }
#define PUT(...) do {                                                         \
        int _r = snprintf(buf + w, w < max ? max - w : 0, __VA_ARGS__);       \
        if (_r > 0) w += (size_t)_r;                                          \
    } while (0)
    PUT("Planner: builtin (%s), %s, member %u of %u", c->plan,
        c->kind ? "reduce" : "allreduce", c->g->my, c->g->size);
    if (c->kind) {
        PUT(", root %u", c->root);
    }
    PUT("\nPhases: %u\n", c->nsteps);
    if (c->rma) {
        PUT(c->rma == RMA_DEV ?
            "Buffers: device memory; remote keys once per op, every step reads its "
            "senders' buffers in one kernel\n" :
            "Buffers: shared memory; remote keys once per op, every step reads its "
            "senders' buffers in place\n");
    }
    for (k = 0; k < c->nsteps; k++) {
        const op_step_t *s = &c->steps[k];
        unsigned e;
        PUT("Step #%u (step_idx %u): %s", k, (unsigned)s->step_idx,
            method_name[s->method]);
        if (s->send_cnt && !s->recv_first) {
            PUT(", send %s to", s->send_recv_buffer ? "recv.buffer" : "send.buffer");
            for (e = 0; e < s->send_cnt; e++) {
                PUT(" %u", s->send_peers[e]);
            }
        }
        if (s->recv_cnt) {
            PUT(", receive from");
            for (e = 0; e < s->recv_cnt; e++) {
                PUT(" %u", s->recv_peers[e]);
            }
        }
        if (s->send_cnt && s->recv_first) {
            PUT(", then send recv.buffer to");
            for (e = 0; e < s->send_cnt; e++) {
                PUT(" %u", s->send_peers[e]);
            }
            if (s->pipelined) {
                PUT(" (pipelined by fragment)");
            }
        }
        if (s->incast) {
            PUT(s->send_cnt ? ", incast (%s packer)" : ", incast", packer_name[s->packer]);
        }
        PUT(", fragment length %zu, fragments per endpoint %llu, "
            "fragments total %llu, aggregation %s\n",
            s->frag_len ? s->frag_len : c->length, (unsigned long long)s->frags,
            (unsigned long long)s->fragments_total,
            s->aggregation == AGG_REDUCE ? "reduce" :
            s->aggregation == AGG_WRITE ? "write" : "nop");
    }
#undef PUT
    return w < max ? w : max - 1;
}
