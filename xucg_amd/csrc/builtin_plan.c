/*
 * builtin_plan.c - the builtin planner's plans for the engine: the tree of
 * builtin/plan/builtin_tree.c (intra-host with its socket level, inter-host of
 * a radix, tree_connect's four phases with waypoints) and recursive K-ing of
 * builtin/plan/builtin_recursive.c (with the host-master hybrid), in the
 * root-first virtual numbering; each step's fragmentation and incast
 * choices (builtin_control.c).
 */
#define _GNU_SOURCE
#include "builtin_int.h"

#include <string.h>

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

/* The virtual numbering for `root`. Hosts are runs of ppn consecutive
 * members (the "by node" allocation builtin_tree.c:397-405 assumes); a layout
 * that is not, as seen from this member, is UCS_ERR_UNSUPPORTED. */
UCG_INTERNAL ucs_status_t plan_ctx_init(ucg_builtin_lgroup_t *g, unsigned root, plan_ctx_t *pc)
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
UCG_INTERNAL ucs_status_t plan_tree(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc, int fanout,
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
UCG_INTERNAL ucs_status_t plan_recursive(ucg_builtin_lcoll_t *c, const plan_ctx_t *pc,
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

UCG_INTERNAL ucs_status_t plan_finish(ucg_builtin_lcoll_t *c, unsigned ppn)
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
                s->incast          = g->incast == 2 ? 2 : 1;
                s->incast_expected = ppn - 1;
                s->fragments_total = s->frags;
            } else if (s->method == M_SEND_TO_SM_ROOT) {
                s->incast          = 1;
                s->incast_expected = ppn - 1;
                s->packer = g->incast == 2 ? PACK_BATCHED :
                            ucg_builtin_combine_atomic_sum_length(g->cmb, c->op, c->dtype)
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
