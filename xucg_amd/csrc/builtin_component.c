/*
 * builtin_component.c - the builtin planner as a UCG plan component.
 *
 * This is the drop-in boundary of the repository: the
 * global `ucg_builtin_component`, of the reference's ucg_plan_component_t
 * (api/ucg_plan_component.h:141-188), defined with UCG_PLAN_COMPONENT_DEFINE
 * under the reference's name, config prefix ("BUILTIN_") and config table
 * (builtin/builtin.c:33-64, 1007-1016). base/ - ucg_plan_query/init
 * (base/ucg_plan.c:72-178), ucg_collective_create/start (base/ucg_group.c:
 * 391-563) - finds it in ucg_plan_components_list and drives it through the
 * vtable; base/ and api/ stay as they are.
 *
 * Behind the vtable is this build's engine (include/ucg_builtin_ops.h): the
 * reference's plans, slots, stash and steps, with every combine going through
 * the combine dispatcher (reduce_cb_f on the host, or the MI355X kernels for
 * device-resident buffers and staged steps), over the shared-memory
 * active-message transport that stands in for the UCT interface of
 * ucg_plan_connect (base/ucg_plan.c:320-439) on one host.
 *
 *   query     builtin.c:231-244 (ucg_plan_single, base/ucg_plan.c:230-243)
 *   init      builtin.c:342-368: the AM id, the config
 *   create    builtin.c:376-456: per-group state, the resend timer
 *   destroy   builtin.c:480-524
 *   plan      builtin.c:533-606 with ucg_builtin_choose_topology :94-131
 *   prepare   ucg_builtin_op_create, builtin_control.c:1106-1282
 *   trigger   ucg_builtin_op_trigger, builtin_control.c:1309-1352
 *   progress  ucg_builtin_op_progress, builtin.c:318-340
 *   discard   ucg_builtin_op_discard, builtin_control.c:1284-1304
 *   print     builtin.c:750-901
 *   fault     builtin.c:1000-1004 (not implemented there either)
 *
 * Built against include/ucg_api_abi.h (this build's declaration of those
 * types, over compat/) by default, or against the reference's own
 * <ucg/api/ucg_plan_component.h> with -DXUCG_REFERENCE_API - the compiler
 * then checks every vtable signature against the reference's types
 * (tests/test_component.py).
 */
#define _GNU_SOURCE
#define UCG_BUILTIN_DEV_HAVE_UCS 1     /* ucs_status_t comes from <ucs/type/status.h> */

#ifdef XUCG_REFERENCE_API
#include <ucg/api/ucg_plan_component.h>
#else
#include "ucg_api_abi.h"
#endif

#include "ucg_builtin_component.h"
#include "ucg_builtin_ops.h"

#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* What base/ defines (ucg_plan.c, ucg_context.c:318) and UCX's parser
 * (ucs_config_global_list): weak here, so that the component also loads on
 * its own (tests, ctypes); the definitions of a loaded base/ take precedence. */
__attribute__((weak)) ucs_list_link_t ucg_plan_components_list =
    UCS_LIST_INITIALIZER(ucg_plan_components_list);
__attribute__((weak)) ucs_list_link_t ucs_config_global_list =
    UCS_LIST_INITIALIZER(ucs_config_global_list);
__attribute__((weak)) ucg_params_t ucg_global_params;

/* ---- configuration (builtin.c:33-64, builtin_plan.h:192-205) ------------ */
typedef struct ucg_builtin_config {
    struct {
        unsigned radix;                /* TREE_RADIX */
        unsigned sock_thresh;          /* TREE_SOCKET_LEVEL_PPN_THRESH */
    } tree;
    struct {
        unsigned factor;               /* RECURSIVE_FACTOR */
    } recursive;
    struct {
        unsigned dimension;            /* NEIGHBOR_DIMENTION (no plan reads it) */
    } neighbor;
    size_t   short_max_tx;             /* the transport's max_short here */
    size_t   bcopy_max_tx;
    unsigned mem_reg_opt_cnt;
    unsigned mem_rma_opt_cnt;
    double   resend_timer_tick;        /* seconds; 0 = no timer thread */
} ucg_builtin_config_t;

static ucs_config_field_t ucg_builtin_tree_table[] = {
    {"RADIX", "8", "Tree radix, for inter-node trees",
     ucs_offsetof(ucg_builtin_config_t, tree.radix) -
     ucs_offsetof(ucg_builtin_config_t, tree), UCS_CONFIG_TYPE_UINT},
    {"SOCKET_LEVEL_PPN_THRESH", "16",
     "From this many members per host on, a second (socket) intra-host level",
     ucs_offsetof(ucg_builtin_config_t, tree.sock_thresh) -
     ucs_offsetof(ucg_builtin_config_t, tree), UCS_CONFIG_TYPE_UINT},
    {NULL}
};

static ucs_config_field_t ucg_builtin_recursive_table[] = {
    {"FACTOR", "2", "Recursive K-ing factor", 0, UCS_CONFIG_TYPE_UINT},
    {NULL}
};

static ucs_config_field_t ucg_builtin_neighbor_table[] = {
    {"DIMENTION", "2", "Neighborhood dimension", 0, UCS_CONFIG_TYPE_UINT},
    {NULL}
};

static ucs_config_field_t ucg_builtin_config_table[] = {
    {"TREE_", "", NULL, ucs_offsetof(ucg_builtin_config_t, tree),
     UCS_CONFIG_TYPE_TABLE(ucg_builtin_tree_table)},
    {"RECURSIVE_", "", NULL, ucs_offsetof(ucg_builtin_config_t, recursive),
     UCS_CONFIG_TYPE_TABLE(ucg_builtin_recursive_table)},
    {"NEIGHBOR_", "", NULL, ucs_offsetof(ucg_builtin_config_t, neighbor),
     UCS_CONFIG_TYPE_TABLE(ucg_builtin_neighbor_table)},
    {"SHORT_MAX_TX_SIZE", "256", "Largest active message, header included",
     ucs_offsetof(ucg_builtin_config_t, short_max_tx), UCS_CONFIG_TYPE_MEMUNITS},
    {"BCOPY_MAX_TX_SIZE", "32768", "Largest send operation to use buffer copy",
     ucs_offsetof(ucg_builtin_config_t, bcopy_max_tx), UCS_CONFIG_TYPE_MEMUNITS},
    {"MEM_REG_OPT_CNT", "10", "Operation counter before registering the memory",
     ucs_offsetof(ucg_builtin_config_t, mem_reg_opt_cnt), UCS_CONFIG_TYPE_UINT},
    {"MEM_RMA_OPT_CNT", "3", "Operation counter before switching to one-sided sends",
     ucs_offsetof(ucg_builtin_config_t, mem_rma_opt_cnt), UCS_CONFIG_TYPE_UINT},
    {"RESEND_TIMER_TICK", "100ms", "Resolution of the (async) resend timer",
     ucs_offsetof(ucg_builtin_config_t, resend_timer_tick), UCS_CONFIG_TYPE_TIME},
    {NULL}
};

/* ---- contexts -------------------------------------------------------------- */
typedef struct ucg_builtin_ctx {
    uint8_t              am_id;
    ucg_builtin_config_t config;
} ucg_builtin_ctx_t;

typedef struct ucg_builtin_group_ctx {
    ucg_builtin_ctx_t        *bctx;
    ucg_group_h               group;
    const ucg_group_params_t *group_params;
    ucg_group_id_t            group_id;
    unsigned                  size;
    unsigned                  my;
    uint8_t                   distance[UCG_BUILTIN_OPS_MAX_MEMBERS];
    ucg_builtin_combine_t    *cmb;
    ucg_builtin_shm_iface_t  *iface;
    ucg_builtin_lgroup_t     *lgroup;
    ucs_list_link_t           plans;       /* for cleanup, builtin.c:512-517 */
} UCS_V_ALIGNED(UCS_SYS_CACHE_LINE_SIZE) ucg_builtin_group_ctx_t;

typedef struct ucg_builtin_plan {
    ucg_plan_t               super;        /* base/ fills it, ucg_group.c:82-100 */
    ucg_builtin_group_ctx_t *gctx;
    int                      kind;         /* 0 allreduce, 1 reduce to root */
    uint16_t                 modifiers;
    ucs_list_link_t          list;         /* in gctx->plans */
    ucs_list_link_t          ops;          /* prepared ops, discarded with it */
} ucg_builtin_plan_t;

typedef struct ucg_builtin_op {
    ucg_op_t                 super;
    ucg_builtin_plan_t      *bplan;
    ucg_builtin_lcoll_t     *lcoll;
    ucs_list_link_t          list;         /* in bplan->ops */
} ucg_builtin_op_t;

extern ucg_plan_component_t ucg_builtin_component;

/* the builtin-private classifier every group's combine gets (SURVEY.md 8b:
 * MAX/MIN/PROD and fp16 vs bf16 cannot be told apart through api/) */
static ucg_builtin_op_classifier_f g_op_cls;
static ucg_builtin_dt_classifier_f g_dt_cls;

void ucg_builtin_component_set_classifier(ucg_builtin_op_classifier_f op_cls,
                                          ucg_builtin_dt_classifier_f dt_cls)
{
    g_op_cls = op_cls;
    g_dt_cls = dt_cls;
}

/* without UCG_PARAM_FIELD_DATATYPE_CB the dtype handle already is a UCP
 * datatype (api/ucg.h:356-361); a contiguous one is (length << 3) */
static int dtype_as_ucp(void *datatype, uintptr_t *ucp_datatype)
{
    *ucp_datatype = (uintptr_t)datatype;
    return 0;
}

/* ---- the vtable ----------------------------------------------------------- */
static ucs_status_t ucg_builtin_query(ucg_plan_desc_t *descs, unsigned *desc_cnt_p)
{
    if (descs) {
        memset(descs, 0, sizeof(*descs));
        descs->component = &ucg_builtin_component;
        snprintf(descs->name, UCG_PLAN_COMPONENT_NAME_MAX, "%s",
                 ucg_builtin_component.name);
        descs->modifiers_supported = (unsigned)-1;   /* builtin.c:239 */
        descs->flags               = 0;
    }
    *desc_cnt_p = 1;
    return UCS_OK;
}

static ucs_status_t ucg_builtin_init(ucg_plan_ctx_h pctx, ucg_plan_params_t *params,
                                     ucg_plan_config_t *config)
{
    ucg_builtin_ctx_t *bctx = pctx;
    if (bctx == NULL || params == NULL || params->am_id == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    bctx->am_id = *params->am_id;
    ++*params->am_id;
    if (config != NULL) {
        memcpy(&bctx->config, config, sizeof(bctx->config));
        return UCS_OK;
    }
    /* no parsed config (a loader without UCX's parser): the environment, as
     * UCX would read it for the table above */
    return ucs_config_parser_fill_opts(&bctx->config, ucg_builtin_config_table,
                                       ucg_builtin_component.config.prefix);
}

static void ucg_builtin_finalize(ucg_plan_ctx_h pctx)
{
    (void)pctx;
}

#define UCG_BUILTIN_PARAM_MASK (UCG_GROUP_PARAM_FIELD_ID | UCG_GROUP_PARAM_FIELD_MEMBER_COUNT | \
                                UCG_GROUP_PARAM_FIELD_MEMBER_INDEX | UCG_GROUP_PARAM_FIELD_DISTANCES)

/* the members of one job and group meet in one shared-memory object */
static void iface_name(char *buf, size_t max, const ucg_group_params_t *p)
{
    unsigned long uid = 0;
    const char *e = getenv("UCX_BUILTIN_JOB_UID");
    if (ucg_global_params.field_mask & UCG_PARAM_FIELD_JOB_UID) {
        uid = ucg_global_params.job_uid;
    } else if (e) {
        uid = strtoul(e, NULL, 0);
    }
    snprintf(buf, max, "/xucg_job%lu_grp%u_n%lu", uid, (unsigned)p->id,
             (unsigned long)p->member_count);
}

static ucs_status_t ucg_builtin_create(ucg_plan_ctx_h pctx, ucg_group_ctx_h ctx,
                                       ucg_group_h group,
                                       const ucg_group_params_t *params)
{
    ucg_builtin_ctx_t *bctx       = pctx;
    ucg_builtin_group_ctx_t *gctx = ctx;
    ucg_builtin_reduce_params_t rp;
    ucg_builtin_combine_config_t ccfg;
    ucg_builtin_lgroup_params_t lp;
    char name[96];
    ucs_status_t st;
    unsigned m;

    if (params == NULL ||
        (params->field_mask & UCG_BUILTIN_PARAM_MASK) != UCG_BUILTIN_PARAM_MASK) {
        return UCS_ERR_INVALID_PARAM;          /* builtin.c:386-389 */
    }
    if (params->member_count == 0 || params->member_count > UCG_BUILTIN_OPS_MAX_MEMBERS ||
        params->member_index >= params->member_count || params->distance == NULL) {
        return UCS_ERR_UNSUPPORTED;
    }
    memset(gctx, 0, sizeof(*gctx));
    gctx->bctx         = bctx;
    gctx->group        = group;
    gctx->group_params = params;
    gctx->group_id     = params->id;
    gctx->size         = (unsigned)params->member_count;
    gctx->my           = (unsigned)params->member_index;
    ucs_list_head_init(&gctx->plans);
    for (m = 0; m < gctx->size; m++) {
        gctx->distance[m] = (uint8_t)params->distance[m];
    }

    /* the MPI library's callbacks, from the process-wide parameters */
    memset(&rp, 0, sizeof(rp));
    rp.reduce_cb_f       = ucg_global_params.reduce_op.reduce_cb_f;
    rp.is_sum_f          = ucg_global_params.reduce_op.is_sum_f;
    rp.is_loc_expected_f = ucg_global_params.reduce_op.is_loc_expected_f;
    rp.is_commutative_f  = ucg_global_params.reduce_op.is_commutative_f;
    if (ucg_global_params.field_mask & UCG_PARAM_FIELD_DATATYPE_CB) {
        rp.convert             = (int (*)(void*, uintptr_t*))ucg_global_params.datatype.convert;
        rp.is_integer_f        = ucg_global_params.datatype.is_integer_f;
        rp.is_floating_point_f = ucg_global_params.datatype.is_floating_point_f;
    } else {
        rp.convert = dtype_as_ucp;
    }
    ucg_builtin_combine_config_read(&ccfg);
    st = ucg_builtin_combine_create(&rp, &ccfg, &gctx->cmb);
    if (st != UCS_OK) {
        return st;
    }
    if (g_op_cls || g_dt_cls) {
        ucg_builtin_combine_set_classifier(gctx->cmb, g_op_cls, g_dt_cls);
    }
    iface_name(name, sizeof(name), params);
    st = ucg_builtin_shm_iface_open(name, gctx->size, gctx->my,
                                    bctx->config.short_max_tx, 64, &gctx->iface);
    if (st != UCS_OK) {
        goto err_cmb;
    }
    lp.distance         = gctx->distance;
    lp.tree_radix       = bctx->config.tree.radix;
    lp.sock_thresh      = bctx->config.tree.sock_thresh;
    lp.recursive_factor = bctx->config.recursive.factor;
    /* the configured BUILTIN_MEM_REG_OPT_CNT (0: never register) */
    lp.mem_reg_opt_cnt  = bctx->config.mem_reg_opt_cnt ? (int)bctx->config.mem_reg_opt_cnt : -1;
    /* The wire header needs a non-zero group id (builtin_control.c:645
     * asserts it); base/ accepts a caller's id 0 (ucg_group.c:302-303). The
     * group's transport object is its own (iface_name), so any non-zero
     * internal id is unique on it. */
    st = ucg_builtin_lgroup_create_ex(gctx->iface, params->id ? params->id : 1, gctx->size,
                                      gctx->my, gctx->cmb, &lp, &gctx->lgroup);
    if (st != UCS_OK) {
        goto err_iface;
    }
    /* ucg_context_set_async_timer(ucg_builtin_async_check), builtin.c:408-413 */
    if (bctx->config.resend_timer_tick > 0.0) {
        st = ucg_builtin_lgroup_set_async_timer(gctx->lgroup,
                                                bctx->config.resend_timer_tick);
        if (st != UCS_OK) {
            goto err_group;
        }
    }
    return UCS_OK;

err_group:
    ucg_builtin_lgroup_destroy(gctx->lgroup);
err_iface:
    (void)ucg_builtin_shm_iface_close(gctx->iface);
err_cmb:
    ucg_builtin_combine_destroy(gctx->cmb);
    return st;
}

static void ucg_builtin_op_discard(ucg_op_t *op);

static void destroy_plan(ucg_builtin_plan_t *plan)
{
    while (!ucs_list_is_empty(&plan->ops)) {
        ucg_builtin_op_t *op = ucs_list_extract_head(&plan->ops, ucg_builtin_op_t, list);
        ucg_builtin_op_discard(&op->super);
    }
    ucs_list_del(&plan->list);
    free(plan);
}

static _Atomic int g_destroy_status = UCS_OK;

ucs_status_t ucg_builtin_component_last_destroy_status(void)
{
    return (ucs_status_t)atomic_load(&g_destroy_status);
}

static void ucg_builtin_destroy(ucg_group_ctx_h ctx)
{
    ucg_builtin_group_ctx_t *gctx = ctx;
    ucs_status_t st;
    while (!ucs_list_is_empty(&gctx->plans)) {
        destroy_plan(ucs_container_of(gctx->plans.next, ucg_builtin_plan_t, list));
    }
    ucg_builtin_lgroup_destroy(gctx->lgroup);    /* stops the resend timer first */
    /* a peer that is gone ends the close with a status, not the process */
    st = ucg_builtin_shm_iface_close(gctx->iface);
    if (st != UCS_OK) {
        fprintf(stderr, "ucg_builtin: group %u member %u: tear-down with status %d "
                "(a member failed)\n", (unsigned)gctx->group_id, gctx->my, (int)st);
    }
    atomic_store(&g_destroy_status, (int)st);
    ucg_builtin_combine_destroy(gctx->cmb);
}

/* ucg_builtin_choose_topology (builtin.c:94-131) restricted to what reduces:
 * SINGLE_DESTINATION + AGGREGATE is MPI_Reduce (the fan-in tree), AGGREGATE
 * alone (with BROADCAST) MPI_Allreduce (recursive or tree, by group size).
 * Fan-out, gather, alltoall and barrier plans carry no combine and are out of
 * this build's scope: UCS_ERR_UNSUPPORTED, so base/ may fall
 * back to another planner. */
static ucs_status_t ucg_builtin_plan(ucg_group_ctx_h ctx,
                                     const ucg_collective_type_t *coll_type,
                                     ucg_plan_t **plan_p)
{
    ucg_builtin_group_ctx_t *gctx = ctx;
    const uint16_t mods = coll_type->modifiers;
    ucg_builtin_plan_t *plan;
    int kind;

    if ((mods & (UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_SOURCE |
                 UCG_GROUP_COLLECTIVE_MODIFIER_CONCATENATE |
                 UCG_GROUP_COLLECTIVE_MODIFIER_BARRIER |
                 UCG_GROUP_COLLECTIVE_MODIFIER_VARIADIC |
                 UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE_PARTIAL |
                 UCG_GROUP_COLLECTIVE_MODIFIER_NEIGHBOR)) ||
        !(mods & UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE)) {
        return UCS_ERR_UNSUPPORTED;
    }
    kind = (mods & UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_DESTINATION) ? 1 : 0;
    if (kind == 1 && coll_type->root >= gctx->size) {
        return UCS_ERR_INVALID_PARAM;
    }
    plan = calloc(1, sizeof(*plan));
    if (plan == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    plan->gctx      = gctx;
    plan->kind      = kind;
    plan->modifiers = mods;
    plan->super.group_id   = gctx->group_id;     /* base/ sets these again */
    plan->super.group_size = gctx->size;
    plan->super.my_index   = gctx->my;
    plan->super.group      = gctx->group;
    ucs_list_head_init(&plan->super.op_head);
    ucs_list_head_init(&plan->ops);
    ucs_list_add_head(&gctx->plans, &plan->list);
    *plan_p = &plan->super;
    return UCS_OK;
}

/* the engine's op for these parameters (ucg_builtin_op_create,
 * builtin_control.c:1106-1282): send.buffer (MPI_IN_PLACE: recv.buffer),
 * recv.buffer, send.count elements of send.dtype, the reduce op in recv.op,
 * the root of a reduce in send.type.root */
static ucs_status_t make_lcoll(ucg_builtin_plan_t *plan, const ucg_collective_params_t *p,
                               ucg_builtin_lcoll_t **lcoll_p)
{
    ucg_builtin_group_ctx_t *gctx = plan->gctx;
    const void *sbuf = p->send.buffer;
    void *rbuf       = p->recv.buffer;
    if ((ucg_global_params.field_mask & UCG_PARAM_FIELD_MPI_IN_PLACE) &&
        sbuf == ucg_global_params.mpi_in_place) {
        sbuf = rbuf;
    }
    if (p->send.count < 0 || p->send.count > 0x7fffffff) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (plan->kind == 0) {
        return ucg_builtin_lcoll_allreduce(gctx->lgroup, sbuf, rbuf, (int)p->send.count,
                                           p->send.dtype, UCG_PARAM_OP(p), lcoll_p);
    }
    return ucg_builtin_lcoll_reduce(gctx->lgroup, sbuf, rbuf, (int)p->send.count,
                                    p->send.dtype, UCG_PARAM_OP(p),
                                    (unsigned)UCG_PARAM_TYPE(p).root, lcoll_p);
}

static ucs_status_t ucg_builtin_op_trigger(ucg_op_t *op, ucg_coll_id_t coll_id,
                                           void *request);

static ucs_status_t ucg_builtin_op_create(ucg_plan_t *plan,
                                          const ucg_collective_params_t *coll_params,
                                          ucg_op_t **new_op)
{
    ucg_builtin_plan_t *bplan = (ucg_builtin_plan_t*)plan;
    ucg_builtin_op_t *op;
    ucs_status_t st;

    if (posix_memalign((void**)&op, UCS_SYS_CACHE_LINE_SIZE, sizeof(*op)) != 0) {
        return UCS_ERR_NO_MEMORY;
    }
    memset(op, 0, sizeof(*op));
    st = make_lcoll(bplan, coll_params, &op->lcoll);
    if (st != UCS_OK) {
        free(op);
        return st;
    }
    /* base/ compares the first cache line of these to reuse the op
     * (base/ucg_group.c:407-431) */
    memcpy(&op->super.params, coll_params, sizeof(*coll_params));
    op->super.trigger_f = ucg_builtin_op_trigger;
    op->super.discard_f = ucg_builtin_op_discard;
    op->super.plan      = plan;
    op->bplan           = bplan;
    ucs_list_add_tail(&bplan->ops, &op->list);
    *new_op = &op->super;
    return UCS_OK;
}

static ucs_status_t ucg_builtin_op_trigger(ucg_op_t *op, ucg_coll_id_t coll_id,
                                           void *request)
{
    ucg_builtin_op_t *bop = (ucg_builtin_op_t*)op;
    ucs_status_t st;
    /* ucg_builtin_comp_last_step_cb (builtin_comp_step.inl:31-32): base/
     * always installs coll_comp_cb_f (ucg_context.c:375-379); the flag and
     * status offsets serve a caller without one */
    st = ucg_builtin_lcoll_set_completion(bop->lcoll,
                                          ucg_global_params.completion.coll_comp_cb_f,
                                          request,
                                          ucg_global_params.completion.comp_flag_offset,
                                          ucg_global_params.completion.comp_status_offset);
    if (st != UCS_OK) {
        return st;
    }
    st = ucg_builtin_lcoll_start_as(bop->lcoll, coll_id);
    /* a busy slot: builtin_control.c:1319-1322 */
    return (st == UCS_ERR_BUSY) ? UCS_ERR_NO_RESOURCE : st;
}

static unsigned ucg_builtin_op_progress(ucg_coll_h coll)
{
    ucg_builtin_op_t *bop = (ucg_builtin_op_t*)coll;
    return ucg_builtin_lgroup_progress(bop->bplan->gctx->lgroup);
}

static void ucg_builtin_op_discard(ucg_op_t *op)
{
    ucg_builtin_op_t *bop = (ucg_builtin_op_t*)op;
    ucs_list_del(&bop->list);
    ucg_builtin_lcoll_destroy(bop->lcoll);
    free(bop);
}

static void ucg_builtin_print(ucg_plan_t *plan, const ucg_collective_params_t *coll_params)
{
    ucg_builtin_plan_t *bplan = (ucg_builtin_plan_t*)plan;
    ucg_builtin_lcoll_t *lcoll;
    char text[4096];

    printf("Planner:       %s\n", ucg_builtin_component.name);
    printf("Collective:    %s, group %u, member %u of %u\n",
           bplan->kind ? "reduce" : "allreduce", (unsigned)bplan->gctx->group_id,
           bplan->gctx->my, bplan->gctx->size);
    if (coll_params == NULL) {
        return;
    }
    /* dry-run the op's creation, as the reference dry-runs step_create */
    if (make_lcoll(bplan, coll_params, &lcoll) != UCS_OK) {
        printf("failed to create the operation for these parameters\n");
        return;
    }
    ucg_builtin_lcoll_describe(lcoll, text, sizeof(text));
    fputs(text, stdout);
    ucg_builtin_lcoll_destroy(lcoll);
}

static ucs_status_t ucg_builtin_handle_fault(ucg_group_ctx_h gctx,
                                             ucg_group_member_index_t index)
{
    (void)gctx;
    (void)index;
    return UCS_ERR_NOT_IMPLEMENTED;
}

UCG_PLAN_COMPONENT_DEFINE(ucg_builtin_component, "builtin",
                          sizeof(ucg_builtin_ctx_t),
                          sizeof(ucg_builtin_group_ctx_t),
                          ucg_builtin_query, ucg_builtin_init,
                          ucg_builtin_finalize, ucg_builtin_create,
                          ucg_builtin_destroy, ucg_builtin_plan,
                          ucg_builtin_op_create, ucg_builtin_op_trigger,
                          ucg_builtin_op_progress, ucg_builtin_op_discard,
                          ucg_builtin_print, ucg_builtin_handle_fault, "BUILTIN_",
                          ucg_builtin_config_table, ucg_builtin_config_t);
