/*
 * builtin_rma.c - remote-key steps of the builtin engine: an op on device
 * buffers (HIP IPC keys, the combine kernels reading peers over xGMI) or on
 * large host messages (POSIX shared-memory keys, reduce_cb_f) runs its plan as
 * READY / DONE control messages around reads of the senders' buffers.
 */
#define _GNU_SOURCE
#include "builtin_int.h"

#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

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
 * dbuf[cur] and writes dbuf[!cur] unless nobody reads dbuf[cur]. A send
 * buffer from the group's registered memory is a third, read-only buffer
 * (index 2) exposed in place of the init copy. The association is the host
 * path's: the accumulator first, then the peers in the order their READYs
 * arrived (builtin_comp_step.inl:213-221). */
#define RMA_DONE 0x40   /* payload {from, buf}: done reading your dbuf[buf] */
#define RMA_RKEY 0x80   /* payload {from, buf, handle}: the key of my dbuf[buf] */
#define RMA_MIN_SHORT (8 + 8 + UCG_BUILTIN_DEV_IPC_HANDLE_BYTES)

struct rma_msg {
    unsigned peer;
    uint64_t header;
    uint32_t length;
    uint8_t  payload[8 + UCG_BUILTIN_DEV_IPC_HANDLE_BYTES];
};


static int rma_trace_on(void);

struct rma_pool {
    void    *ptr;
    size_t   bytes;
    int      kind;
    int      busy;
    int      user;            /* handed out by ucg_builtin_lgroup_mem_alloc */
    int      in_arena;        /* carved out of the group's device arena */
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

/* segments of processes that died before their group was destroyed (a
 * killed worker): removed once per process, before its first segment */
static void shm_seg_sweep(void)
{
    static _Atomic int done;
    DIR *d;
    struct dirent *e;
    if (atomic_exchange(&done, 1) || (d = opendir("/dev/shm")) == NULL) {
        return;
    }
    while ((e = readdir(d)) != NULL) {
        char path[300];
        int pid;
        unsigned q;
        if (sscanf(e->d_name, "xucg_rma_%d_%u", &pid, &q) == 2 && pid > 0 &&
            kill(pid, 0) != 0 && errno == ESRCH) {
            snprintf(path, sizeof(path), "/%s", e->d_name);
            shm_unlink(path);
        }
    }
    closedir(d);
}

static void *shm_seg_alloc(size_t bytes, void *key)
{
    static _Atomic unsigned seq;
    shm_key_t k;
    void *p;
    int fd;
    shm_seg_sweep();
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
    struct stat sb;
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
    /* a key that claims more than the segment holds would fault on access */
    if (fstat(fd, &sb) != 0 || (uint64_t)sb.st_size < k.bytes || k.bytes == 0) {
        close(fd);
        return UCS_ERR_INVALID_PARAM;
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

/* UCX_BUILTIN_DEV_POOL_BYTES (default 32 MiB, 0 = none): the device arena
 * out of which a group's registered buffers are carved while it lasts. It is
 * made on the group's first device-buffer (remote-key) buffer, not with the
 * group: a group that never runs a device-buffer step costs no HBM (ADVICE
 * r04). arena_bytes holds the size still to make while arena is NULL. */
/* the arena, once; a failure is reported once and leaves the group without
 * one (a member whose arena failed silently took per-buffer
 * allocations while its peers did not) */
static void rma_arena_make(ucg_builtin_lgroup_t *g)
{
    if (g->arena != NULL || g->arena_bytes == 0) {
        return;
    }
    g->arena = ucg_builtin_combine_dev_alloc(g->cmb, g->arena_bytes);
    if (g->arena == NULL) {
        fprintf(stderr, "ucg_builtin: group %u member %u: the %zu B device arena "
                "(UCX_BUILTIN_DEV_POOL_BYTES) could not be allocated (%s); its "
                "registered buffers are allocated one by one\n", (unsigned)g->group_id,
                g->my, g->arena_bytes, ucg_builtin_dev_last_error());
        g->arena_bytes = 0;
    }
}

/* UCX_BUILTIN_DEV_POOL_EAGER=y makes the arena with the group, so that the
 * first device-buffer operation pays no allocation (a hipMalloc of 32 MiB
 * may synchronise the device) */
UCG_INTERNAL void rma_group_init(ucg_builtin_lgroup_t *g)
{
    const size_t bytes = parse_memunits(getenv("UCX_BUILTIN_DEV_POOL_BYTES"),
                                        (size_t)32 << 20);
    const char *eager = getenv("UCX_BUILTIN_DEV_POOL_EAGER");
    g->arena = NULL;
    g->arena_used = 0;
    g->arena_bytes = (bytes && ucg_builtin_combine_has_device(g->cmb)) ? bytes : 0;
    if (eager && (eager[0] == 'y' || eager[0] == '1')) {
        rma_arena_make(g);
    }
}

/* registered buffers come in size classes - at least 64 KiB, eight per
 * power of two (at most 12.5 % over the request) - so that ops of many
 * different sizes share buffers: pool memory is never returned before the
 * group is destroyed (peers keep their mappings, keyed by the buffer's key) */
static size_t rma_pool_class(size_t bytes)
{
    size_t c = bytes < ((size_t)64 << 10) ? ((size_t)64 << 10) : bytes, step;
    unsigned lg = 0;
    while (((size_t)2 << lg) <= c) {
        lg++;
    }
    step = (size_t)1 << (lg - 3);
    return (c + step - 1) / step * step;
}

/* the smallest free registered buffer that holds `bytes` and is less than
 * twice its class, or a new one of the class */
static int rma_pool_get(ucg_builtin_lgroup_t *g, size_t bytes, int kind)
{
    const size_t cls = rma_pool_class(bytes);
    struct rma_pool *p;
    unsigned i;
    int best = -1;
    for (i = 0; i < g->npool; i++) {
        if (!g->pool[i].busy && g->pool[i].kind == kind && g->pool[i].bytes >= cls &&
            g->pool[i].bytes < 2 * cls &&
            (best < 0 || g->pool[i].bytes < g->pool[best].bytes)) {
            best = (int)i;
        }
    }
    if (best >= 0) {
        g->pool[best].busy = 1;
        return best;
    }
    bytes = cls;
    p = realloc(g->pool, (g->npool + 1) * sizeof(*p));
    if (p == NULL) {
        return -1;
    }
    g->pool = p;
    p = &g->pool[g->npool];
    p->bytes    = bytes;
    p->kind     = kind;
    p->busy     = 1;
    p->user     = 0;
    p->in_arena = 0;
    if (kind == RMA_SHM) {
        p->ptr = shm_seg_alloc(bytes, p->key);
        return p->ptr ? (int)g->npool++ : -1;
    }
    /* the group's first device buffer: make the arena now */
    rma_arena_make(g);
    if (g->arena && g->arena_used + bytes <= g->arena_bytes) {
        /* from the group's arena: one allocation per group, not one per
         * buffer, and the peers map the whole arena once (one key, offsets) */
        p->ptr = (char*)g->arena + g->arena_used;
        p->in_arena = 1;
        g->arena_used += bytes;
    } else {
        p->ptr = ucg_builtin_combine_dev_alloc(g->cmb, bytes);
        if (p->ptr == NULL) {
            return -1;
        }
    }
    if (ucg_builtin_combine_dev_export(g->cmb, p->ptr, p->key) != UCS_OK) {
        if (!p->in_arena) {
            ucg_builtin_combine_dev_free(g->cmb, p->ptr);
        } else {
            g->arena_used -= bytes;
        }
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
        if (rma_trace_on()) {
            fprintf(stderr, "[rma %u] import of member %u's buffer failed (%d): %s\n", g->my,
                    peer, (int)st, kind == RMA_SHM ? "shared memory" : ucg_builtin_dev_last_error());
        }
        return st;
    }
    if (rma_trace_on()) {
        fprintf(stderr, "[rma %u] import of member %u's buffer -> %p\n", g->my, peer, *ptr);
    }
    m = &g->imp[g->nimp++];
    m->peer = peer;
    m->kind = kind;
    memcpy(m->key, key, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
    m->ptr = *ptr;
    return UCS_OK;
}

/* Group destroy is collective but not synchronised: a peer may still map this
 * member's pool buffers when they are given back here. Pool buffers and the
 * arena are exported device memory - hipMalloc memory with hipIpc keys by
 * default, shareable allocations with UCX_BUILTIN_DEV_POOL_MEM=shareable. A
 * free retires their keys, so a later group can never map them by an old key.
 * Plain memory then goes to the process's reuse cache (the same memory at the
 * same address, which keeps the runtime's hipIpc mappings right, DESIGN.md
 * 7), shareable memory back to the device (a peer's mapping holds it). A
 * buffer rma_free left taken - an op that ended before every peer was done
 * (a timeout, an error, a destroy while running) - may still be read by a
 * peer: it is parked instead, never handed out again, and so is the arena
 * when such a buffer lies in it. Shared-memory segments stay
 * alive for the peers that map them. */
UCG_INTERNAL void rma_group_free(ucg_builtin_lgroup_t *g)
{
    unsigned i;
    int park_arena = 0;
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
            /* taken by an op (rma_free keeps a buffer with readers taken) */
            const int readers = g->pool[i].busy && !g->pool[i].user;
            if (g->pool[i].in_arena) {
                park_arena |= readers;
            } else if (readers) {
                ucg_builtin_combine_dev_park(g->cmb, g->pool[i].ptr);
            } else {
                ucg_builtin_combine_dev_free(g->cmb, g->pool[i].ptr);
            }
        }
    }
    if (g->arena) {
        if (park_arena) {
            ucg_builtin_combine_dev_park(g->cmb, g->arena);
        } else {
            ucg_builtin_combine_dev_free(g->cmb, g->arena);
        }
        g->arena = NULL;
    }
    free(g->imp);
    free(g->pool);
}

/* UCX_BUILTIN_SHM_ZCOPY_THRESH: host messages of at least this many bytes
 * take the shared-memory remote-key steps (0 or unset = never; this build's
 * knob - the reference hard-codes 100000, builtin_control.c:474) */
static size_t shm_zcopy_thresh(void)
{
    return parse_memunits(getenv("UCX_BUILTIN_SHM_ZCOPY_THRESH"), 0);
}

/* the op's buffers decide: device memory (both, or the one given) ->
 * RMA_DEV, large host messages with the knob -> RMA_SHM, other host
 * memory -> 0, one of each -> -1 */
UCG_INTERNAL int rma_kind(ucg_builtin_lgroup_t *g, const void *sbuf, const void *rbuf,
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

/* a device call of this op that blocked for seconds (a key import, the
 * first launch of a kernel, a fold) is named on stderr: peers waiting on this
 * member time out meanwhile, and the note says where it stood */
static ucs_status_t slow_note(const ucg_builtin_lcoll_t *c, const char *what, double t0,
                              ucs_status_t st)
{
    const double dt = now_s() - t0;
    if (dt > 2.0) {
        struct timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        fprintf(stderr, "[ucg slow] member %u coll_id %u: %s took %.1f s (status %d), "
                "ended at %.3f\n", c->g->my, c->coll_id, what, dt, (int)st,
                ts.tv_sec + ts.tv_nsec * 1e-9);
    }
    return st;
}

/* XUCG_RMA_TRACE=1: every device write of the remote-key steps (its dst
 * range and its sources), every pool buffer and every imported peer buffer,
 * one line each on stderr - so that a corrupted range in a test can be matched
 * against what the engine wrote */
static int rma_trace_on(void)
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("XUCG_RMA_TRACE");
        on = e && (e[0] == '1' || e[0] == 'y');
    }
    return on;
}

static void rma_trace(const ucg_builtin_lcoll_t *c, const char *what, const void *dst,
                      size_t bytes, const void *const *srcs, unsigned n)
{
    unsigned i;
    if (!rma_trace_on()) {
        return;
    }
    fprintf(stderr, "[rma %u c%u] %s dst %p..%p", c->g->my, c->coll_id, what, dst,
            (const void*)((const char*)dst + bytes));
    for (i = 0; i < n; i++) {
        fprintf(stderr, "%s%p", i ? " " : " src ", srcs[i]);
    }
    fputc('\n', stderr);
}

/* the receive's combine: dst = srcs[n-1] (op) (... (srcs[1] (op) srcs[0])) */
static ucs_status_t rma_fold(ucg_builtin_lcoll_t *c, void *dst, const void *const *srcs,
                             unsigned n)
{
    unsigned m;
    ucs_status_t st = UCS_OK;
    if (ops_on_timer_thread()) {
        c->g->async_combines++;         /* a15: the fold on the resend timer */
    }
    if (c->rma == RMA_DEV) {
        const double t0 = now_s();
        rma_trace(c, "fold", dst, c->length, srcs, n);
        return slow_note(c, "fold", t0,
                         ucg_builtin_combine_dev_fold(c->g->cmb, c->op, c->dtype, dst,
                                                      srcs, n, (size_t)c->count));
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

/* buffer b of this member: dbuf 0 / 1, or 2 = the registered send.buffer */
static void *rma_local(const ucg_builtin_lcoll_t *c, unsigned b)
{
    return b == 2 ? (void*)c->sbuf : c->dbuf[b];
}

static ucs_status_t rma_copy(ucg_builtin_lcoll_t *c, void *dst, const void *src)
{
    if (c->rma == RMA_DEV) {
        const double t0 = now_s();
        rma_trace(c, "copy", dst, c->length, &src, 1);
        return slow_note(c, "copy", t0,
                         ucg_builtin_combine_dev_copy(c->g->cmb, dst, src, c->length));
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

    /* the receive half starts once this member's messages are out: the
     * reference's step sends all it has before draining what came in
     * (ucg_builtin_step_execute, then check_pending: builtin_data.c:584-668,
     * builtin_comp_step.inl:403-462). Sends stopped at UCS_ERR_NO_RESOURCE
     * resume from progress or from the resend timer (builtin.c:260-294),
     * which then folds on its own thread. */
    if (c->rdy_cnt[k] < s->recv_cnt || c->send_pending) {
        return 0;
    }
    if (c->cur_buf == 2) {
        out = c->readers[0] ? 1 : 0;      /* never written: the caller's send buffer */
    } else {
        out = c->readers[c->cur_buf] ? !c->cur_buf : c->cur_buf;
    }
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
        srcs[0] = rma_local(c, c->cur_buf);
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

/* ---- recursive doubling on device buffers as one exchange ----------------
 * For an allreduce whose plan is plain recursive doubling (a power-of-two
 * group on one host, factor 2), every element of the result is
 * V(self, log2 N) of builtin_recursive.c:158-169 - the same on every member.
 * On device buffers the whole plan then runs as two remote-key phases over
 * all xGMI links at once instead of log2 N pairwise ones: (0) every member
 * exposes its data and computes its 1/N shard of V with one kernel reading
 * that shard from all N buffers (ucg_builtin_dev_reduce_multi); (1) every
 * member exposes its reduced shard and copies all N shards into recv.buffer.
 * A small message (oneshot 2) skips phase 1: phase 0 reads all of every
 * member's buffer and writes the whole of V into recv.buffer. Same bits as
 * the steps; UCX_BUILTIN_DEVICE_ONESHOT=n runs the steps. From 4 to 16
 * members (reduce_multi's operand limit). A small allreduce over a one-host
 * tree (oneshot 3) is the same single pass with the root's fold. */
static int oneshot_enabled(int kind)
{
    const char *e = getenv(kind == RMA_DEV ? "UCX_BUILTIN_DEVICE_ONESHOT" :
                                             "UCX_BUILTIN_SHM_ONESHOT");
    return !(e && (e[0] == 'n' || e[0] == 'N' || e[0] == '0'));
}

/* messages up to this size skip the all-gather: every member evaluates the
 * whole of V(self) from all N buffers in one kernel, straight into
 * recv.buffer (N x the reads, one launch and one wait less). On host memory
 * the N x reads are reduce_cb_f work on every member's core and lost on
 * every size measured, so there it is off unless asked for. */
static size_t oneshot_full_bytes(int kind)
{
    return kind == RMA_DEV ?
           parse_memunits(getenv("UCX_BUILTIN_DEVICE_ONESHOT_FULL"), (size_t)1 << 20) :
           parse_memunits(getenv("UCX_BUILTIN_SHM_ONESHOT_FULL"), 0);
}

/* The two-phase one-shot gives every member the same bits: shard r is V(r)
 * on every member. The steps give member s V(s) everywhere, and V(r) and V(s)
 * differ where the op does not commute bit for bit on the data: on floats,
 * two NaNs of different payloads in SUM / PROD (which payload survives follows
 * the operand order), and MAX / MIN of MPI's (dst > src) ? dst : src form
 * meeting NaN or +0 / -0 (builtin_recursive.c:158-169 fixes the operand
 * order per member). Integer ops commute exactly. Which NaN payload a SUM
 * keeps is not even fixed by the reference: `b[i] = a[i] + b[i]` in the MPI
 * library may compile with either operand first. MAX / MIN's comparison is
 * fixed by the source. So UCX_BUILTIN_ONESHOT_FLOAT_SPLIT = "sum" (the
 * default) splits float SUM / PROD, "y" every float op, "n" none; a float op
 * that may not split runs the single pass (V(self) on every member, exact)
 * below the single-pass limit and the plan's steps above it. */
static int oneshot_split_allowed(ucg_builtin_lcoll_t *c)
{
    const char *e = getenv("UCX_BUILTIN_ONESHOT_FLOAT_SPLIT");
    ucg_dev_op_t o;
    ucg_dev_dtype_t d;
    if (!ucg_builtin_combine_classify(c->g->cmb, c->op, c->dtype, &o, &d)) {
        return 0;                       /* unknown: assume it may not commute */
    }
    if (d != UCG_DEV_DT_FLOAT16 && d != UCG_DEV_DT_BFLOAT16 &&
        d != UCG_DEV_DT_FLOAT32 && d != UCG_DEV_DT_FLOAT64) {
        return 1;
    }
    if (e && (e[0] == 'y' || e[0] == 'Y' || e[0] == '1')) {
        return 1;
    }
    if (e && (e[0] == 'n' || e[0] == 'N' || e[0] == '0')) {
        return 0;
    }
    return o == UCG_DEV_OP_SUM || o == UCG_DEV_OP_PROD;
}

/* dst = V(self, log2 N) of srcs[0..N) (member r's data at srcs[r]) over n
 * elements: the device kernel, or on host memory the same tree of
 * reduce_cb_f calls (level h folds val[m + h] into val[m], val[m] holding
 * member self ^ m), the first level into dst and scratch */
static ucs_status_t rma_butterfly(ucg_builtin_lcoll_t *c, void *dst, const void *const *srcs,
                                  unsigned N, unsigned self, size_t n)
{
    const size_t bytes = n * c->dt_len;
    const void *val[16];
    unsigned h, m;
    ucs_status_t st = UCS_OK;
    if (ops_on_timer_thread()) {
        c->g->async_combines++;
    }
    if (c->rma == RMA_DEV) {
        const double t0 = now_s();
        rma_trace(c, "butterfly", dst, bytes, srcs, N);
        return slow_note(c, "butterfly", t0,
                         ucg_builtin_combine_dev_butterfly(c->g->cmb, c->op, c->dtype, dst,
                                                           srcs, N, self, n));
    }
    if (n == 0) {
        return UCS_OK;
    }
    if (N > 2 && c->bf_bytes < (N / 2 - 1) * bytes) {
        void *p = realloc(c->bf_scratch, (N / 2 - 1) * bytes);
        if (p == NULL) {
            return UCS_ERR_NO_MEMORY;
        }
        c->bf_scratch = p;
        c->bf_bytes   = (N / 2 - 1) * bytes;
    }
    for (m = 0; m < N; m++) {
        val[m] = srcs[self ^ m];
    }
    for (h = 1; h < N && st == UCS_OK; h <<= 1) {
        for (m = 0; m < N && st == UCS_OK; m += 2 * h) {
            void *acc = (void*)val[m];
            if (h == 1) {
                acc = m ? (char*)c->bf_scratch + (m / 2 - 1) * bytes : dst;
                memcpy(acc, val[m], bytes);
            }
            st = ucg_builtin_combine_reduce(c->g->cmb, c->op, (void*)val[m + h], acc,
                                            (int)n, c->dtype);
            val[m] = acc;
        }
    }
    return st;
}

/* dsts[i][0:bytes] = srcs[i][0:bytes] for every i */
static ucs_status_t rma_copy_n(ucg_builtin_lcoll_t *c, void *const *dsts,
                               const void *const *srcs, unsigned k, size_t bytes)
{
    unsigned i;
    if (c->rma == RMA_DEV) {
        const double t0 = now_s();
        for (i = 0; i < k; i++) {
            rma_trace(c, "copy_n", dsts[i], bytes, &srcs[i], 1);
        }
        return slow_note(c, "copy_n", t0,
                         ucg_builtin_combine_dev_copy_n(c->g->cmb, dsts, srcs, k, bytes));
    }
    for (i = 0; i < k; i++) {
        memcpy(dsts[i], srcs[i], bytes);
    }
    return UCS_OK;
}

/* every other member on this host and, below the socket-level threshold or
 * without sockets, at one level: the intra-host tree of a one-host group is
 * then member 0 with all others as children (every member sees the same, as
 * the planner assumes symmetric layouts) */
static int flat_host_tree(const ucg_builtin_lgroup_t *g)
{
    unsigned m;
    for (m = 0; m < g->size; m++) {
        const uint8_t d = g->distance[m];
        if (m == g->my) {
            continue;
        }
        if (d > D_HOST || d < D_SOCKET || (d == D_SOCKET && g->size >= g->sock_thresh)) {
            return 0;
        }
    }
    return 1;
}

/* shard r of the op: [r * se, min(count, (r + 1) * se)) elements, se a
 * multiple of 256 bytes so shards start on 256-B boundaries */
static void oneshot_shard(const ucg_builtin_lcoll_t *c, unsigned r, size_t *lo, size_t *n)
{
    const size_t per = 256 / c->dt_len ? 256 / c->dt_len : 1;
    const size_t cnt = (size_t)c->count, N = c->g->size;
    size_t se = (cnt + N - 1) / N;
    se = (se + per - 1) / per * per;
    *lo = (size_t)r * se < cnt ? (size_t)r * se : cnt;
    *n  = (*lo + se < cnt ? *lo + se : cnt) - *lo;
}

/* phase 0 exposes this member's data (dbuf 0, or the registered send
 * buffer), phase 1 its reduced shard in dbuf 1 */
static unsigned oneshot_buf(const ucg_builtin_lcoll_t *c, unsigned phase)
{
    return phase ? 1 : (c->exp_sbuf ? 2 : 0);
}

static void oneshot_expose(ucg_builtin_lcoll_t *c, unsigned phase)
{
    const unsigned b = oneshot_buf(c, phase);
    unsigned p;
    for (p = 0; p < c->g->size; p++) {
        if (p != c->g->my) {
            rma_post(c, p, (uint8_t)(phase + 1), b, NULL, 0);
        }
    }
    c->readers[b] += c->g->size - 1;
}

/* the phase's kernel once every peer's READY is in; DONE to all */
static int oneshot_receive(ucg_builtin_lcoll_t *c, unsigned phase)
{
    const unsigned N = c->g->size, my = c->g->my;
    const void *srcs[16];
    const void *peer[16];               /* each member's exposed buffer */
    void *dsts[16];
    ucs_status_t st = UCS_OK;
    size_t lo, n, full_lo, full_n;
    unsigned r, k, i;

    if (c->rdy_cnt[phase] < N - 1 || c->send_pending) {
        return 0;                       /* see rma_receive */
    }
    peer[my] = rma_local(c, oneshot_buf(c, phase));
    for (i = 0; i < N - 1; i++) {
        r = c->rdy_peer[phase][i];
        peer[r] = c->peer_buf[r][c->rdy_buf[phase][i]];
        if (peer[r] == NULL) {
            finish(c, UCS_ERR_IO_ERROR);          /* a READY without a key */
            return 0;
        }
    }
    if (c->oneshot == 3) {
        /* ucg_builtin_step_recv_handle_chunk at the tree's root, member 0:
         * its data first, then every child's (builtin_comp_step.inl:213-221) */
        st = rma_fold(c, c->rbuf_user, peer, N);
    } else if (phase == 0 && c->oneshot == 2) {
        for (r = 0; r < N; r++) {
            srcs[r] = peer[r];
        }
        st = rma_butterfly(c, c->rbuf_user, srcs, N, my, (size_t)c->count);
    } else if (phase == 0) {
        oneshot_shard(c, my, &lo, &n);
        for (r = 0; r < N; r++) {
            srcs[r] = (const char*)peer[r] + lo * c->dt_len;
        }
        st = rma_butterfly(c, (char*)c->dbuf[1] + lo * c->dt_len, srcs, N, my, n);
    } else {
        /* every full shard in one launch, the ragged last one in another */
        oneshot_shard(c, 0, &full_lo, &full_n);
        for (k = 0, r = 0; r < N && st == UCS_OK; r++) {
            oneshot_shard(c, r, &lo, &n);
            if (n == 0) {
                continue;
            }
            srcs[k] = (const char*)peer[r] + lo * c->dt_len;
            dsts[k] = c->rbuf_user + lo * c->dt_len;
            if (n != full_n) {
                st = rma_copy_n(c, &dsts[k], &srcs[k], 1, n * c->dt_len);
            } else {
                k++;
            }
        }
        if (st == UCS_OK) {
            st = rma_copy_n(c, dsts, srcs, k, full_n * c->dt_len);
        }
    }
    if (st != UCS_OK) {
        finish(c, st);
        return 0;
    }
    for (i = 0; i < N - 1; i++) {
        rma_post(c, c->rdy_peer[phase][i], RMA_DONE, c->rdy_buf[phase][i], NULL, 0);
    }
    return 1;
}

static void oneshot_advance(ucg_builtin_lcoll_t *c)
{
    const unsigned phases = c->oneshot >= 2 ? 1 : 2;
    while (!c->done && c->cur < phases) {
        if (!c->rma_sent) {
            oneshot_expose(c, c->cur);
            c->rma_sent = 1;
        }
        if (!oneshot_receive(c, c->cur)) {
            return;
        }
        c->cur++;
        c->rma_sent = 0;
    }
    c->rma_final = 1;                 /* phase 1 wrote recv.buffer */
}

/* as far as the messages in allow; the op completes once the result is in
 * recv.buffer and nobody reads this member's buffers any more */
UCG_INTERNAL void rma_advance(ucg_builtin_lcoll_t *c)
{
    if (c->rma_busy) {
        c->rma_again = 1;
        return;
    }
    c->rma_busy = 1;
    do {
        c->rma_again = 0;
        rma_flush(c);
        if (c->oneshot) {
            oneshot_advance(c);
        }
        while (!c->oneshot && !c->done && c->cur < c->nsteps) {
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
                rma_copy(c, c->rbuf_user, rma_local(c, c->cur_buf)) : UCS_OK;
            if (st != UCS_OK) {
                finish(c, st);
            }
            c->rma_final = 1;
        }
        rma_flush(c);
        if (!c->done && c->rma_final && c->out_tail == 0 &&
            c->readers[0] == 0 && c->readers[1] == 0 && c->readers[2] == 0) {
            finish(c, UCS_OK);
        }
    } while (c->rma_again && !c->done);
    c->rma_busy = 0;
}

/* a control message of this op (am_handler, or the stash at start) */
UCG_INTERNAL void rma_msg(ucg_builtin_lcoll_t *c, ops_header_t h, const void *data,
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
    if (w[0] >= c->g->size || w[0] == c->g->my || w[1] > 2) {
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
        const double t0 = now_s();
        st = slow_note(c, "key import", t0,
                       rma_import(c->g, w[0], c->rma, (const char*)data + 8, &p));
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
    } else if (c->oneshot) {
        k = h.step_idx - 1u;              /* phases 0 (buffer 0 or 2) and 1 */
        if (k > 1 || (w[1] == 1) != (k == 1) || c->rdy_cnt[k] == c->g->size - 1) {
            finish(c, UCS_ERR_IO_ERROR);
            return;
        }
        c->rdy_peer[k][c->rdy_cnt[k]] = (uint8_t)w[0];
        c->rdy_buf[k][c->rdy_cnt[k]]  = (uint8_t)w[1];
        c->rdy_cnt[k]++;
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
UCG_INTERNAL ucs_status_t rma_setup(ucg_builtin_lcoll_t *c, void *rbuf_user)
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
    /* from 4 members on: at 2 the one step moves no more than the exchange
     * (r02os: 64 MiB, 0.187 ms one-shot against 0.127 ms as the step) */
    c->oneshot   = c->kind == 0 && oneshot_enabled(c->rma) &&
                   c->g->size >= 4 && c->g->size <= 16 && c->plan &&
                   strcmp(c->plan, "recursive doubling") == 0;
    if (c->oneshot && c->length <= oneshot_full_bytes(c->rma)) {
        c->oneshot = 2;
    } else if (c->oneshot && !oneshot_split_allowed(c)) {
        c->oneshot = 0;
    }
    /* a one-host allreduce tree is flat (tree_add_intra: every member's parent
     * is member 0), so a small message runs as one pass too: the root's fold,
     * children in index order - one arrival order the steps may see */
    if (!c->oneshot && c->kind == 0 && oneshot_enabled(c->rma) &&
        c->g->size >= 3 && c->g->size <= 16 &&
        c->length <= oneshot_full_bytes(c->rma) && c->plan && strcmp(c->plan, "tree") == 0 &&
        flat_host_tree(c->g)) {
        c->oneshot = 3;
    }
    for (i = 0; i < 2; i++) {
        int k = rma_pool_get(c->g, c->length ? c->length : 1, c->rma);
        if (k < 0) {
            return UCS_ERR_NO_MEMORY;
        }
        c->pool_idx[i] = k;
        c->dbuf[i]     = c->g->pool[k].ptr;
        if (rma_trace_on()) {
            fprintf(stderr, "[rma %u] op buffer %u: pool %d %p..%p\n", c->g->my, i, k,
                    c->g->pool[k].ptr,
                    (void*)((char*)c->g->pool[k].ptr + c->g->pool[k].bytes));
        }
        memcpy(c->key[i], c->g->pool[k].key, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
    }
    /* a send buffer the caller took from the group's registered memory is
     * exposed where it is (the zcopy send of a registered buffer,
     * builtin_control.c:276-286, 943-949); in place it is written at the end,
     * so it is copied as any other */
    c->exp_sbuf = 0;
    for (i = 0; c->sbuf && c->sbuf != c->rbuf_user && i < c->g->npool; i++) {
        const struct rma_pool *p = &c->g->pool[i];
        if (p->user && p->kind == c->rma && p->ptr == (const void*)c->sbuf &&
            p->bytes >= c->length) {
            c->exp_sbuf = 1;
            memcpy(c->key[2], p->key, UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
            break;
        }
    }
    return UCS_OK;
}

UCG_INTERNAL ucs_status_t rma_start(ucg_builtin_lcoll_t *c, op_slot_t *slot)
{
    ucs_status_t st;
    unsigned k, e;
    stash_t **pp;

    c->cur       = 0;
    c->cur_buf   = 0;
    c->rma_sent  = c->rma_recvd = c->rma_final = 0;
    c->readers[0] = c->readers[1] = c->readers[2] = 0;
    c->out_head  = c->out_tail = 0;
    c->send_pending = 0;
    memset(c->rdy_cnt, 0, sizeof(c->rdy_cnt));
    if (c->length == 0) {
        c->status = UCS_OK;
        lcoll_set_done(c);
        lcoll_notify(c);
        return UCS_OK;
    }
    /* ucg_builtin_init_reduce (builtin_control.c:43-47): this member's data
     * into its first buffer - every member, since every member exposes it -
     * unless the send buffer is registered and exposed in place */
    c->cur_buf = c->exp_sbuf ? 2 : 0;
    st = c->exp_sbuf ? UCS_OK : rma_copy(c, c->dbuf[0], c->sbuf ? c->sbuf : c->rbuf);
    if (st != UCS_OK) {
        c->status = st;
        lcoll_set_done(c);
        lcoll_notify(c);
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
        for (k = 0; k < (c->oneshot ? 1 : c->nsteps); k++) {
            const unsigned ne = c->oneshot ? c->g->size : c->steps[k].send_cnt;
            for (e = 0; e < ne; e++) {
                unsigned p = c->oneshot ? e : c->steps[k].send_peers[e];
                if (p == c->g->my) {
                    continue;
                }
                if (!sent[p]) {
                    sent[p] = 1;
                    rma_post(c, p, RMA_RKEY, 0, c->key[0], UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
                    rma_post(c, p, RMA_RKEY, 1, c->key[1], UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
                    if (c->exp_sbuf) {
                        rma_post(c, p, RMA_RKEY, 2, c->key[2],
                                 UCG_BUILTIN_DEV_IPC_HANDLE_BYTES);
                    }
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

/* the op's buffers go back to the group's pool; peers' mappings stay. A
 * buffer that peers may still be reading - the op ended before every DONE
 * came back (destroyed while running, a timeout, an error) - stays taken
 * until the group is destroyed, so that no later op writes it under them */
UCG_INTERNAL void rma_free(ucg_builtin_lcoll_t *c)
{
    unsigned i;
    for (i = 0; i < 2; i++) {
        if (c->pool_idx[i] >= 0 && c->readers[i] == 0) {
            c->g->pool[c->pool_idx[i]].busy = 0;
        }
    }
    free(c->outbox);
    free(c->bf_scratch);
}

/* ---- registered group memory ------------------------------------------- */
void *ucg_builtin_lgroup_mem_alloc(ucg_builtin_lgroup_t *g, size_t bytes, int on_device)
{
    const int kind = on_device ? RMA_DEV : RMA_SHM;
    int k;
    if (g == NULL || bytes == 0 ||
        (on_device && !ucg_builtin_combine_has_device(g->cmb))) {
        return NULL;
    }
    /* the pool is the group's: an op starting or resent on the timer's
     * thread takes buffers from it under the same lock */
    void *ptr = NULL;
    pthread_mutex_lock(g->async_lock);
    k = rma_pool_get(g, bytes, kind);
    if (k >= 0) {
        g->pool[k].user = 1;
        ptr = g->pool[k].ptr;       /* the table may grow once unlocked */
    }
    pthread_mutex_unlock(g->async_lock);
    return ptr;
}

void ucg_builtin_lgroup_mem_free(ucg_builtin_lgroup_t *g, void *ptr)
{
    unsigned i;
    if (g == NULL || ptr == NULL) {
        return;
    }
    pthread_mutex_lock(g->async_lock);
    for (i = 0; i < g->npool; i++) {
        if (g->pool[i].user && g->pool[i].ptr == ptr) {
            g->pool[i].user = 0;      /* back to the pool: the memory and its key */
            g->pool[i].busy = 0;      /* stay valid until the group is destroyed */
            break;
        }
    }
    pthread_mutex_unlock(g->async_lock);
}
