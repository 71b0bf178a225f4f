/*
 * builtin_ops.c - the builtin planner's operation engine around the combine
 * (include/ucg_builtin_ops.h): receive slots, the stash, step execution and
 * completion, the SM-root packers, and the group / collective API.
 *
 * This is a C restatement of the receive/step machinery of the reference's
 * builtin/ops (file:line anchors at each function), written against this
 * build's combine dispatcher instead of a direct reduce_cb_f call. With the
 * transport of builtin_shm.c, the plans of builtin_plan.c and the
 * remote-key steps of builtin_rma.c, it runs the reference's allreduce and
 * reduce plans end to end between processes with no UCX underneath.
 */
#define _GNU_SOURCE
#include "builtin_int.h"

#include <fcntl.h>
#include <sched.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

static const char *const packer_name[] = {"copy", "reducing", "atomic", "batched"};
static const char *const method_name[] = {
    "REDUCE_RECURSIVE", "REDUCE_TERMINAL", "SEND_TO_SM_ROOT", "SEND_TERMINAL",
    "RECV_TERMINAL", "REDUCE_WAYPOINT", "BCAST_WAYPOINT"
};

static int  recv_cb(ucg_builtin_lcoll_t *c, uint64_t offset, const void *data,
                    size_t length);
static void step_execute(ucg_builtin_lcoll_t *c);

/* set on the resend timer's thread: what it combines is counted */
static __thread int on_timer_thread;

UCG_INTERNAL int ops_on_timer_thread(void)
{
    return on_timer_thread;
}

/* UCS_ASYNC_BLOCK / UNBLOCK of the group (recursive: completion callbacks and
 * the stash drain re-enter the engine on the same thread) */
static inline void group_block(ucg_builtin_lgroup_t *g)
{
    pthread_mutex_lock(g->async_lock);
}

static inline void group_unblock(ucg_builtin_lgroup_t *g)
{
    pthread_mutex_unlock(g->async_lock);
}

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

/* finish the op: ucg_builtin_comp_last_step_cb, builtin_comp_step.inl:8-38.
 * An op this member gives up on (any error not caused by a peer) is published
 * (shm_abandon), so that its peers end it with UCS_ERR_CANCELED instead of
 * waiting for messages that never come (group_check_peers). */
UCG_INTERNAL void finish(ucg_builtin_lcoll_t *c, ucs_status_t status)
{
    op_slot_t *slot = &c->g->slots[c->coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT];
    if (c->step_open) {
        ucs_status_t st = ucg_builtin_combine_step_end(c->g->cmb);
        if (status == UCS_OK) {
            status = st;
        }
        c->step_open = 0;
    }
    if (status != UCS_OK && c->active && !c->peer_ended) {
        shm_abandon(c->g->iface, c->g->group_id,
                    abandon_word(c->g->gen, c->g->group_id, c->seq));
    }
    c->status       = status;
    lcoll_set_done(c);
    c->active       = 0;
    c->send_pending = 0;
    c->step_started = 0;
    slot->req       = NULL;
    slot->expecting = 0;
    lcoll_notify(c);
}

/* coll_comp_cb_f, or the completion flag and status in the request
 * (ucg_builtin_comp_last_step_cb, builtin_comp_step.inl:31-32) */
UCG_INTERNAL void lcoll_notify(ucg_builtin_lcoll_t *c)
{
    if (!c->comp_set) {
        return;
    }
    if (c->comp_cb) {
        c->comp_cb(c->comp_req, c->status);
    } else {
        ucs_status_t st = c->status;
        memcpy((char*)c->comp_req + c->comp_status_off, &st, sizeof(st));
        *((volatile uint8_t*)c->comp_req + c->comp_flag_off) = 1;
    }
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
    if (s->packer == PACK_BATCHED) {
        return ucg_builtin_shm_am_incast_batched(c->g->iface, peer, header,
                                                 s->incast_expected, buf, n);
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
                c->staged_dev |= ucg_builtin_combine_step_on_device(g->cmb);
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

    if (s->incast == 2 && s->aggregation == AGG_REDUCE) {
        /* BATCHED_DATA (builtin_comp_step.inl:242-273): one message carries
         * every child's chunk for this offset, each behind its own header;
         * they are reduced into the same range in record order. The
         * reference computes dest_buffer before it scales the offset (:320
         * against :261-263), so its chunks land at the unscaled offset; here
         * remote_offset is in bytes and every chunk lands where it belongs. */
        const size_t rec = (length + 8) / s->incast_expected;
        const size_t n   = rec - 8;
        unsigned k;
        if (rec * s->incast_expected != length + 8 || rec <= 8 || offset + n > c->length) {
            st = UCS_ERR_IO_ERROR;
        }
        for (k = 0; k < s->incast_expected && st == UCS_OK; k++) {
            const char *chunk = (const char*)data + k * rec;
            if (on_timer_thread) {
                c->g->async_combines++;
            }
            st = c->step_open ?
                 ucg_builtin_combine_fragment(c->g->cmb, offset, chunk, n) :
                 ucg_builtin_combine_reduce(c->g->cmb, c->op, (void*)chunk,
                                            c->rbuf + offset, (int)(n / c->dt_len),
                                            c->dtype);
        }
    } else if (offset + length > c->length) {
        st = UCS_ERR_IO_ERROR;          /* a message outside recv.buffer */
    } else if (s->aggregation == AGG_REDUCE) {
        if (on_timer_thread) {
            c->g->async_combines++;
        }
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

/* BUILTIN_MEM_REG_OPT_CNT (builtin.c:49-50) from the environment, 0 = never
 * register; a group's parameters override it */
static unsigned mem_reg_opt_cnt_env(void)
{
    static unsigned v = (unsigned)-1;
    if (v == (unsigned)-1) {
        v = env_uint("UCX_BUILTIN_MEM_REG_OPT_CNT", 10);
    }
    return v;
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
    g = calloc(1, sizeof(*g));
    if (g == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    /* the other groups' timers may be delivering into the table and the
     * unexpected list right now */
    pthread_mutex_lock(&iface->async_lock);
    if (iface->groups[group_id % UNEXP_GROUPS] != NULL) {
        pthread_mutex_unlock(&iface->async_lock);
        free(g);
        return UCS_ERR_BUSY;
    }
    pthread_cond_init(&g->timer_cv, NULL);
    g->async_lock = &iface->async_lock;
    g->iface    = iface;
    g->group_id = group_id;
    g->size     = member_count;
    g->my       = my_index;
    g->cmb      = combine;
    {
        const char *e = getenv("UCX_BUILTIN_SM_INCAST");
        g->incast = (e && (e[0] == 'b' || e[0] == 'B')) ? 2 :
                    (e && (e[0] == 'y' || e[0] == 'Y' || e[0] == '1'));
        if (g->incast == 2 && !iface->incast_batched) {
            g->incast = 1;     /* the iface was opened without batched cells */
        }
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
    g->mem_reg_opt_cnt = (params && params->mem_reg_opt_cnt) ?
                         (params->mem_reg_opt_cnt < 0 ? 0u : (unsigned)params->mem_reg_opt_cnt) :
                         mem_reg_opt_cnt_env();
    rma_group_init(g);
    g->gen = ++iface->group_gen[group_id % UNEXP_GROUPS];
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
    pthread_mutex_unlock(&iface->async_lock);
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
    if (g->timer_on) {
        /* ucg_context_unset_async_timer, builtin.c:485 */
        group_block(g);
        g->timer_stop = 1;
        pthread_cond_signal(&g->timer_cv);
        group_unblock(g);
        pthread_join(g->timer, NULL);
        g->timer_on = 0;
    }
    /* out of the table first: another group's timer delivers nothing more
     * here once it is gone */
    group_block(g);
    g->iface->groups[g->group_id % UNEXP_GROUPS] = NULL;
    for (i = 0; i < UCG_BUILTIN_OPS_MAX_CONCURRENT; i++) {
        stash_t *m;
        while ((m = g->slots[i].msgs) != NULL) {
            g->slots[i].msgs = m->next;
            free(m);
        }
    }
    group_unblock(g);
    rma_group_free(g);
    pthread_cond_destroy(&g->timer_cv);
    free(g);
}

/* the resend queue (ucg_builtin_async_resend, builtin.c:270-282): every op
 * whose sends stopped at UCS_ERR_NO_RESOURCE goes on from where it stopped; a
 * step whose sends complete drains what is stashed for it, so this may
 * combine. Called with the group blocked. */
static unsigned group_resend(ucg_builtin_lgroup_t *g)
{
    unsigned i, n = 0;
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

/* Peer failure: every op still running ends with a status
 * once a member of the iface is gone (UCS_ERR_CONNECTION_RESET: what it sent
 * before it went was delivered first, a dead process adds nothing more) or a
 * peer published that it gave up on the same op (UCS_ERR_CANCELED) - the
 * reference's error completion, recv_handle_error, builtin_comp_step.inl:
 * 332-333, where a UCX endpoint error would end the request. At most every
 * PEER_CHECK_S, from a waiter or the timer; called with the group blocked. */
static void group_check_peers(ucg_builtin_lgroup_t *g)
{
    ucg_builtin_shm_iface_t *it = g->iface;
    const double t = now_s();
    unsigned i, m;
    int dead;
    if (t - g->peer_check_t < PEER_CHECK_S) {
        return;
    }
    g->peer_check_t = t;
    if ((dead = shm_peer_check(it)) >= 0) {
        (void)ucg_builtin_shm_progress(it, am_handler, it);
    }
    for (i = 0; i < UCG_BUILTIN_OPS_MAX_CONCURRENT; i++) {
        ucg_builtin_lcoll_t *c = g->slots[i].req;
        ucs_status_t st = UCS_OK;
        if (c == NULL || c->done) {
            continue;
        }
        if (dead >= 0) {
            st = UCS_ERR_CONNECTION_RESET;
        } else {
            const uint64_t w = abandon_word(g->gen, g->group_id, c->seq);
            for (m = 0; m < g->size; m++) {
                if (m != g->my && shm_abandoned(it, m, g->group_id) == w) {
                    fprintf(stderr, "ucg_builtin: member %u gave up on collective %u of "
                            "group %u; ending it here\n", m, c->coll_id, g->group_id);
                    st = UCS_ERR_CANCELED;
                    break;
                }
            }
        }
        if (st != UCS_OK) {
            c->peer_ended = 1;
            finish(c, st);
        }
    }
}

/* ucg_builtin_op_progress, builtin.c:318-340: the transport first, then the
 * resend queue; a member that keeps finding nothing looks at its peers */
unsigned ucg_builtin_lgroup_progress(ucg_builtin_lgroup_t *g)
{
    unsigned n;
    group_block(g);
    n  = ucg_builtin_shm_progress(g->iface, am_handler, g->iface);
    n += group_resend(g);
    if (n == 0 && (++g->idle_polls & 1023) == 0) {
        group_check_peers(g);
    }
    group_unblock(g);
    return n;
}

/* ucg_builtin_async_check, builtin.c:284-294, on a timer of its own thread
 * (the UCS async context's timer, set in ucg_builtin_create, :408-413) */
static void *async_timer(void *arg)
{
    ucg_builtin_lgroup_t *g = arg;
    on_timer_thread = 1;
    group_block(g);
    while (!g->timer_stop) {
        struct timespec ts;
        const double t = now_s() + g->timer_tick;   /* CLOCK_MONOTONIC, as the condvar */
        ts.tv_sec  = (time_t)t;
        ts.tv_nsec = (long)((t - (double)(time_t)t) * 1e9);
        pthread_cond_timedwait(&g->timer_cv, g->async_lock, &ts);
        if (!g->timer_stop) {
            g->async_resends += group_resend(g);
            group_check_peers(g);
        }
    }
    group_unblock(g);
    return NULL;
}

ucs_status_t ucg_builtin_lgroup_set_async_timer(ucg_builtin_lgroup_t *g, double interval_s)
{
    pthread_condattr_t a;
    if (g == NULL || interval_s <= 0.0 || g->timer_on) {
        return UCS_ERR_INVALID_PARAM;
    }
    /* the timed wait runs on the monotonic clock, like now_s() */
    pthread_cond_destroy(&g->timer_cv);
    pthread_condattr_init(&a);
    pthread_condattr_setclock(&a, CLOCK_MONOTONIC);
    pthread_cond_init(&g->timer_cv, &a);
    pthread_condattr_destroy(&a);
    g->timer_tick = interval_s;
    g->timer_stop = 0;
    if (pthread_create(&g->timer, NULL, async_timer, g) != 0) {
        return UCS_ERR_NO_RESOURCE;
    }
    g->timer_on = 1;
    return UCS_OK;
}

void ucg_builtin_lgroup_async_stats(ucg_builtin_lgroup_t *g, uint64_t out[2])
{
    out[0] = g ? g->async_resends : 0;
    out[1] = g ? g->async_combines : 0;
}

void ucg_builtin_lgroup_stats(ucg_builtin_lgroup_t *g, uint64_t out[4])
{
    int i;
    if (g == NULL) {
        memset(out, 0, 4 * sizeof(uint64_t));
        return;
    }
    /* under the group's lock: the resend timer's thread counts too (a race
     * ThreadSanitizer found, round 6) */
    group_block(g);
    for (i = 0; i < 4; i++) {
        out[i] = g->stats[i];
    }
    group_unblock(g);
}

static void lcoll_free(ucg_builtin_lcoll_t *c)
{
    if (c && c->rbuf_reg) {
        ucg_builtin_combine_mem_dereg(c->g->cmb, c->rbuf);   /* discard, :1289-1292 */
    }
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
    c->status = UCS_OK;
    lcoll_set_done(c);
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

static ucs_status_t lcoll_allreduce(ucg_builtin_lgroup_t *g, const void *sbuf,
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

static ucs_status_t lcoll_reduce(ucg_builtin_lgroup_t *g, const void *sbuf,
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

ucs_status_t ucg_builtin_lcoll_allreduce(ucg_builtin_lgroup_t *g, const void *sbuf,
                                         void *rbuf, int count, void *dtype,
                                         void *op, ucg_builtin_lcoll_t **coll_p)
{
    ucs_status_t st;
    if (g == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    group_block(g);
    st = lcoll_allreduce(g, sbuf, rbuf, count, dtype, op, coll_p);
    group_unblock(g);
    return st;
}

ucs_status_t ucg_builtin_lcoll_reduce(ucg_builtin_lgroup_t *g, const void *sbuf,
                                      void *rbuf, int count, void *dtype,
                                      void *op, unsigned root,
                                      ucg_builtin_lcoll_t **coll_p)
{
    ucs_status_t st;
    if (g == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    group_block(g);
    st = lcoll_reduce(g, sbuf, rbuf, count, dtype, op, root, coll_p);
    group_unblock(g);
    return st;
}

static ucs_status_t lcoll_start_at(ucg_builtin_lcoll_t *c, uint8_t coll_id);

ucs_status_t ucg_builtin_lcoll_start(ucg_builtin_lcoll_t *c)
{
    ucs_status_t st;
    if (c == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    group_block(c->g);
    st = lcoll_start_at(c, c->g->next_coll_id);
    group_unblock(c->g);
    return st;
}

ucs_status_t ucg_builtin_lcoll_start_as(ucg_builtin_lcoll_t *c, uint8_t coll_id)
{
    ucs_status_t st;
    if (c == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    group_block(c->g);
    st = lcoll_start_at(c, coll_id);
    group_unblock(c->g);
    return st;
}

/* ucg_builtin_op_trigger, builtin_control.c:1309-1352, for the coll_id that
 * ucg_collective_trigger hands out (base/ucg_group.c:485-500) */
static ucs_status_t lcoll_start_at(ucg_builtin_lcoll_t *c, uint8_t coll_id)
{
    ucg_builtin_lgroup_t *g = c->g;
    op_slot_t *slot;

    if (c->active) {
        return UCS_ERR_BUSY;
    }
    slot = &g->slots[coll_id % UCG_BUILTIN_OPS_MAX_CONCURRENT];
    if (slot->req != NULL) {
        return UCS_ERR_BUSY;    /* more than 16 ops outstanding */
    }
    c->coll_id      = coll_id;
    g->next_coll_id = (uint8_t)(coll_id + 1);
    c->seq          = ++g->starts;
    c->peer_ended   = 0;
    if (c->rma) {
        return rma_start(c, slot);
    }
    /* the op's optimisation countdown (ucg_builtin_comp_last_step_cb,
     * builtin_comp_step.inl:24-27 -> ucg_builtin_optimize, builtin_control.c:
     * 345-373): after MEM_REG_OPT_CNT starts that staged a step on the device,
     * its recv buffer is registered, so that every later step's H2D and D2H
     * of it move by DMA */
    if (c->staged_dev && !c->rbuf_reg && c->length &&
        ++c->dev_starts == g->mem_reg_opt_cnt &&
        ucg_builtin_dev_mem_kind(c->rbuf) == UCG_DEV_MEM_HOST &&
        ucg_builtin_combine_mem_reg(g->cmb, c->rbuf, c->length) == UCS_OK) {
        c->rbuf_reg = 1;
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
        c->status = UCS_OK;
        lcoll_set_done(c);
        lcoll_notify(c);
        return UCS_OK;
    }
    c->active = 1;
    slot->req = c;
    step_execute(c);
    return c->done ? c->status : UCS_INPROGRESS;
}

int ucg_builtin_lcoll_test(ucg_builtin_lcoll_t *c, ucs_status_t *status)
{
    const int done = lcoll_is_done(c);
    if (done && status) {
        *status = c->status;
    }
    return done;
}

/* UCX_BUILTIN_TIMEOUT_DUMP=y: on a timed-out wait, the op's state and what
 * sits in the group's stash, on stderr (a diagnosis aid) */
static void timeout_dump(const ucg_builtin_lcoll_t *c)
{
    const ucg_builtin_lgroup_t *g = c->g;
    const char *e = getenv("UCX_BUILTIN_TIMEOUT_DUMP");
    unsigned k, n = 0;
    if (!(e && (e[0] == 'y' || e[0] == '1'))) {
        return;
    }
    fprintf(stderr, "[ucg timeout] member %u coll_id %u plan %s rma %d oneshot %d cur %u/%u "
            "cur_buf %u readers %u/%u/%u rdy %u/%u/%u final %d sent %d recvd %d "
            "outbox %u..%u pending %d stats %llu/%llu/%llu/%llu\n",
            g->my, c->coll_id, c->plan ? c->plan : "-", c->rma, c->oneshot, c->cur,
            c->nsteps, c->cur_buf, c->readers[0], c->readers[1], c->readers[2],
            c->rdy_cnt[0], c->rdy_cnt[1], c->rdy_cnt[2], c->rma_final, c->rma_sent,
            c->rma_recvd, c->out_head, c->out_tail, c->send_pending,
            (unsigned long long)g->stats[0], (unsigned long long)g->stats[1],
            (unsigned long long)g->stats[2], (unsigned long long)g->stats[3]);
    for (k = 0; k < UCG_BUILTIN_OPS_MAX_CONCURRENT; k++) {
        const stash_t *m;
        for (m = g->slots[k].msgs; m && n < 64; m = m->next, n++) {
            ops_header_t h;
            uint32_t w[2] = {0, 0};
            h.header = m->header;
            memcpy(w, m->data, m->length < 8 ? m->length : 8);
            fprintf(stderr, "[ucg timeout]   stashed slot %u coll_id %u step_idx 0x%x "
                    "from %u buf %u len %zu\n", k, h.coll_id, h.step_idx, w[0], w[1],
                    m->length);
        }
    }
}

ucs_status_t ucg_builtin_lcoll_wait(ucg_builtin_lcoll_t *c)
{
    static double lim = -1.0;
    static long spin = -1;
    unsigned idle = 0, busy = 0;
    double t0 = now_s();
    if (lim < 0.0) {
        const char *e = getenv("UCX_BUILTIN_WAIT_SPIN");
        lim  = wait_timeout_s();
        spin = e ? atol(e) : 4096;
    }
    while (!lcoll_is_done(c)) {
        if (ucg_builtin_lgroup_progress(c->g) != 0) {
            idle = 0;
            /* progress counts resend attempts too: a peer that stopped
             * taking messages (its op ended with an error, its process is
             * gone) keeps it non-zero, so the peers and the time limit are
             * checked here as well */
            if ((++busy & 4095) != 0) {
                continue;
            }
            group_block(c->g);
            group_check_peers(c->g);
            group_unblock(c->g);
            if (now_s() - t0 > lim) {
                idle = (unsigned)spin;
            } else {
                continue;
            }
        }
        /* a peer's message is usually a few hundred ns away: spin first,
         * give the core away only when the wait gets long */
        if (++idle < (unsigned long)spin) {
            __builtin_ia32_pause();
            continue;
        }
        if (now_s() - t0 > lim) {
            group_block(c->g);
            if (!c->done) {
                timeout_dump(c);
                finish(c, UCS_ERR_TIMED_OUT);
            }
            group_unblock(c->g);
            break;
        }
        group_block(c->g);
        group_check_peers(c->g);
        group_unblock(c->g);
        sched_yield();
    }
    return c->status;
}

ucs_status_t ucg_builtin_lcoll_set_completion(ucg_builtin_lcoll_t *c,
                                              ucg_builtin_coll_comp_cb_f cb, void *req,
                                              size_t flag_offset, size_t status_offset)
{
    if (c == NULL || c->active || (cb == NULL && req == NULL)) {
        return UCS_ERR_INVALID_PARAM;
    }
    c->comp_set        = 1;
    c->comp_cb         = cb;
    c->comp_req        = req;
    c->comp_flag_off   = flag_offset;
    c->comp_status_off = status_offset;
    return UCS_OK;
}

void ucg_builtin_lcoll_destroy(ucg_builtin_lcoll_t *c)
{
    ucg_builtin_lgroup_t *g;
    if (c == NULL) {
        return;
    }
    g = c->g;
    group_block(g);
    if (c->active) {
        finish(c, UCS_ERR_CANCELED);
    }
    lcoll_free(c);
    group_unblock(g);
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
        if (c->oneshot == 1) {
            PUT("Executed as: one-shot reduce-scatter (every shard of the plan's "
                "association read from all members) + all-gather\n");
        } else if (c->oneshot == 2) {
            PUT("Executed as: one-shot, every member evaluating the plan's association "
                "over all members' data\n");
        } else if (c->oneshot == 3) {
            PUT("Executed as: one-shot, every member folding all members' data as the "
                "tree's root does (children in index order)\n");
        }
        if (c->exp_sbuf) {
            PUT("Send buffer: registered group memory, exposed in place\n");
        }
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
            PUT(s->send_cnt ? ", incast (%s packer)" : s->incast == 2 ? ", incast (batched)" :
                ", incast", packer_name[s->packer]);
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
