/*
 * component_test.c - drives `ucg_builtin_component` through its vtable the
 * way UCG's base/ does, with no UCX underneath: a minimal stand-in for
 * base/ucg_plan.c (component lookup in ucg_plan_components_list, config read,
 * query, init) and base/ucg_group.c (group create, plan cache, op cache by
 * the first 64 bytes of the parameters, trigger with base's coll_id,
 * progress through ucg_request_get_progress, destroy). Test infrastructure.
 *
 *   RANK=r WORLD_SIZE=n MASTER_PORT=p component_test [layout|host|device]
 *   RANK=r WORLD_SIZE=n MASTER_PORT=p component_test latency [iters [count]]
 *
 * Built twice (tests/test_component.py): over this build's declaration of
 * the API (include/ucg_api_abi.h, linked with libucg_builtin.so), and with
 * -DXUCG_REFERENCE_API over the reference's unchanged api/ headers (compat/
 * for the UCX types), linked with builtin_component.c built the same way.
 * "layout" prints the offset and size of every field the component and base/
 * exchange: the two builds must print the same. "host" runs allreduce and
 * reduce ops on host buffers (the combine on reduce_cb_f); "device" on GPU
 * buffers (remote-key steps, the combine kernels), with the builtin-private
 * classifier registered. "latency" times BASELINE config 1 through the
 * vtable. Inputs are exact integers, so every association gives the same
 * bits and the expected result is a plain sum / max.
 */
#define _GNU_SOURCE
#ifdef XUCG_REFERENCE_API
#include <ucg/api/ucg_plan_component.h>
#include <ucg/api/ucg_mpi.h>
#else
#include "ucg_api_abi.h"
#endif
#include "ucg_builtin_component.h"
#include "ucg_builtin_dev.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

UCS_STATIC_ASSERT(sizeof(ucg_collective_params_t) == 64);
UCS_STATIC_ASSERT(offsetof(ucg_op_t, params) % 64 == 0);
UCS_STATIC_ASSERT(sizeof(ucg_collective_type_t) == 8);
UCS_STATIC_ASSERT(sizeof(enum ucg_group_member_distance) == 1);

/* ---- what base/ defines ---------------------------------------------------- */
UCS_LIST_HEAD(ucg_plan_components_list);
UCS_LIST_HEAD(ucs_config_global_list);
ucg_params_t ucg_global_params;

/* ---- the "MPI library" behind reduce_cb_f --------------------------------- */
typedef struct { int id; } mpi_op_t;        /* 0 SUM, 1 MAX */
typedef struct { int size, is_float; } mpi_dt_t;
static mpi_op_t OP_SUM = {0}, OP_MAX = {1};
static mpi_dt_t DT_I32 = {4, 0}, DT_I64 = {8, 0}, DT_F32 = {4, 1}, DT_F64 = {8, 1};

#define LOOP(T)                                                                \
    for (i = 0; i < count; i++) {                                              \
        T a = ((T*)src)[i], b = ((T*)dst)[i];                                  \
        ((T*)dst)[i] = o->id == 0 ? (T)(a + b) : (b > a ? b : a);              \
    }

static int mpi_reduce(void *op, char *src, char *dst, unsigned count, void *dtype)
{
    const mpi_op_t *o = op;
    const mpi_dt_t *d = dtype;
    unsigned i;
    if (d->is_float) {
        if (d->size == 4) { LOOP(float) } else { LOOP(double) }
    } else if (d->size == 4) {
        for (i = 0; i < count; i++) {       /* wraps as MPI's int SUM does */
            uint32_t a = ((uint32_t*)src)[i], b = ((uint32_t*)dst)[i];
            int32_t sa = (int32_t)a, sb = (int32_t)b;
            ((uint32_t*)dst)[i] = o->id == 0 ? a + b : (uint32_t)(sb > sa ? sb : sa);
        }
    } else {
        LOOP(int64_t)
    }
    return 0;
}

static int is_sum(void *op) { return ((mpi_op_t*)op)->id == 0; }
static int no_loc(void *op) { (void)op; return 0; }
static int commutes(void *op) { (void)op; return 1; }
static int convert(void *dt, ucp_datatype_t *u) { *u = (ucp_datatype_t)((mpi_dt_t*)dt)->size << 3; return 0; }
static int is_int(void *dt, int *s) { *s = 1; return !((mpi_dt_t*)dt)->is_float; }
static int is_fp(void *dt) { return ((mpi_dt_t*)dt)->is_float; }
/* the builtin-private classifier: device enums for the ops and types above */
static int op_cls(void *op) { return ((mpi_op_t*)op)->id == 0 ? UCG_DEV_OP_SUM : UCG_DEV_OP_MAX; }
static int dt_cls(void *dt)
{
    const mpi_dt_t *d = dt;
    return d->is_float ? (d->size == 4 ? UCG_DEV_DT_FLOAT32 : UCG_DEV_DT_FLOAT64) :
                         (d->size == 4 ? UCG_DEV_DT_INT32 : UCG_DEV_DT_INT64);
}

typedef struct {
    int           done;
    ucs_status_t  status;
    int           calls;
} request_t;

/* may run on the resend timer's thread (builtin.c:284-294): the status is
 * published by the release store, and the poller reads it after an acquire */
static void comp_cb(void *req, ucs_status_t status)
{
    request_t *r = req;
    r->status = status;
    r->calls++;
    __atomic_store_n(&r->done, 1, __ATOMIC_RELEASE);
}

static char in_place_marker;

/* ---- base/ stand-in ------------------------------------------------------ */
struct ucg_group {
    ucg_group_params_t       params;
    enum ucg_group_member_distance distance[64];
    ucg_plan_desc_t          desc;
    void                    *pctx;
    void                    *gctx;
    ucg_plan_t              *cache[1 << 6];
    ucg_coll_id_t            next_coll_id;
};

static ucg_plan_component_t *find_component(const char *name)
{
    ucg_plan_component_t *c;
    ucs_list_for_each(c, &ucg_plan_components_list, list) {
        if (!strcmp(c->name, name)) {
            return c;
        }
    }
    return NULL;
}

static ucg_collective_params_t last_params;

/* ucg_collective_create, base/ucg_group.c:391-483 (api/ucg.h:431-433; the
 * reference's api/ucg_mpi.h helpers call it) */
ucs_status_t ucg_collective_create(ucg_group_h g, const ucg_collective_params_t *p,
                                   ucg_coll_h *coll)
{
    ucg_plan_component_t *comp = g->desc.component;
    const unsigned key = UCG_PARAM_TYPE(p).modifiers & 0x3f;
    ucg_plan_t *plan = g->cache[key];
    ucg_op_t *op;
    ucs_status_t st;
    memcpy(&last_params, p, sizeof(*p));
    if (plan != NULL) {
        ucs_list_for_each(op, &plan->op_head, list) {
            if (memcmp(p, &op->params, 64) == 0) {
                ucs_list_del(&op->list);
                *coll = op;
                return UCS_OK;
            }
        }
    } else {
        st = comp->plan(g->gctx, &UCG_PARAM_TYPE(p), &plan);
        if (st != UCS_OK) {
            return st;
        }
        ucs_recursive_spinlock_init(&plan->lock, 0);
        plan->my_index   = g->params.member_index;
        plan->group_size = g->params.member_count;
        ucs_list_head_init(&plan->op_head);
        plan->group_id   = g->params.id;
        plan->planner    = &g->desc;
        plan->group      = g;
        g->cache[key]    = plan;
    }
    st = comp->prepare(plan, p, &op);
    if (st == UCS_OK) {
        *coll = op;
    }
    return st;
}

/* ucg_collective_destroy: back into the plan's op cache */
static void coll_destroy(ucg_coll_h coll)
{
    ucg_op_t *op = coll;
    ucs_list_add_head(&op->plan->op_head, &op->list);
}

/* ucg_collective_start + progress until the request completes */
static ucs_status_t coll_run(ucg_group_h g, ucg_coll_h coll)
{
    ucg_op_t *op = coll;
    request_t req = {0, UCS_INPROGRESS, 0};
    /* ucg_request_get_progress, base/ucg_group.c:381-384 */
    ucg_collective_progress_t progress = op->plan->planner->component->progress;
    ucs_status_t st = op->trigger_f(op, g->next_coll_id++, &req);
    const time_t t0 = time(NULL);
    unsigned polls = 0;
    if (st != UCS_OK && st != UCS_INPROGRESS) {
        return st;
    }
    while (!__atomic_load_n(&req.done, __ATOMIC_ACQUIRE)) {
        progress(coll);
        if ((++polls & 4095) == 0 && time(NULL) - t0 > 60) {
            return UCS_ERR_TIMED_OUT;
        }
    }
    if (req.calls != 1 || (st == UCS_OK && req.status != UCS_OK)) {
        fprintf(stderr, "completion callback: %d calls, status %d\n", req.calls, req.status);
        return UCS_ERR_IO_ERROR;
    }
    return req.status;
}

/* ---- layout of everything base/ and the component exchange --------------- */
#define OFF(T, f) printf("offsetof(%s, %s) %zu\n", #T, #f, offsetof(T, f))
#define SZ(T)     printf("sizeof(%s) %zu\n", #T, sizeof(T))
#define VAL(e)    printf("%s %ld\n", #e, (long)(e))

static void dump_layout(void)
{
    SZ(ucg_params_t);
    OFF(ucg_params_t, field_mask); OFF(ucg_params_t, job_uid);
    OFF(ucg_params_t, address.lookup_f); OFF(ucg_params_t, address.release_f);
    OFF(ucg_params_t, neighbors.vertex_count_f); OFF(ucg_params_t, neighbors.vertex_query_f);
    OFF(ucg_params_t, datatype.convert); OFF(ucg_params_t, datatype.is_integer_f);
    OFF(ucg_params_t, datatype.is_floating_point_f);
    OFF(ucg_params_t, reduce_op.reduce_cb_f); OFF(ucg_params_t, reduce_op.is_sum_f);
    OFF(ucg_params_t, reduce_op.is_loc_expected_f);
    OFF(ucg_params_t, reduce_op.is_commutative_f);
    OFF(ucg_params_t, completion.coll_comp_cb_f);
    OFF(ucg_params_t, completion.comp_flag_offset);
    OFF(ucg_params_t, completion.comp_status_offset);
    OFF(ucg_params_t, mpi_in_place); OFF(ucg_params_t, fault.mode);
    OFF(ucg_params_t, fault.context); OFF(ucg_params_t, fault.handler_f);
    OFF(ucg_params_t, fault.err_str_f);
    SZ(ucg_collective_type_t);
    SZ(ucg_group_params_t);
    OFF(ucg_group_params_t, field_mask); OFF(ucg_group_params_t, id);
    OFF(ucg_group_params_t, member_count); OFF(ucg_group_params_t, member_index);
    OFF(ucg_group_params_t, cb_context); OFF(ucg_group_params_t, distance);
    SZ(ucg_collective_params_t);
    OFF(ucg_collective_params_t, send.type); OFF(ucg_collective_params_t, send.buffer);
    OFF(ucg_collective_params_t, send.count); OFF(ucg_collective_params_t, send.dtype);
    OFF(ucg_collective_params_t, recv.op); OFF(ucg_collective_params_t, recv.displs);
    OFF(ucg_collective_params_t, recv.buffer); OFF(ucg_collective_params_t, recv.counts);
    OFF(ucg_collective_params_t, recv.dtypes);
    SZ(ucg_plan_plogp_params_t);
    SZ(ucg_plan_desc_t);
    OFF(ucg_plan_desc_t, component); OFF(ucg_plan_desc_t, modifiers_supported);
    OFF(ucg_plan_desc_t, flags); OFF(ucg_plan_desc_t, latency_estimator);
    OFF(ucg_plan_desc_t, fault_tolerance_supported);
    SZ(ucg_plan_params_t);
    SZ(ucg_plan_t);
    OFF(ucg_plan_t, op_head); OFF(ucg_plan_t, planner); OFF(ucg_plan_t, group_id);
    OFF(ucg_plan_t, group_size); OFF(ucg_plan_t, my_index); OFF(ucg_plan_t, group);
    OFF(ucg_plan_t, priv);
    SZ(ucg_op_t);
    OFF(ucg_op_t, discard_f); OFF(ucg_op_t, list); OFF(ucg_op_t, queue);
    OFF(ucg_op_t, pending_req); OFF(ucg_op_t, plan); OFF(ucg_op_t, params);
    OFF(ucg_op_t, priv);
    SZ(ucg_plan_component_t);
    OFF(ucg_plan_component_t, config); OFF(ucg_plan_component_t, config.prefix);
    OFF(ucg_plan_component_t, config.table); OFF(ucg_plan_component_t, config.size);
    OFF(ucg_plan_component_t, global_ctx_size);
    OFF(ucg_plan_component_t, per_group_ctx_size); OFF(ucg_plan_component_t, list);
    OFF(ucg_plan_component_t, query); OFF(ucg_plan_component_t, init);
    OFF(ucg_plan_component_t, finalize); OFF(ucg_plan_component_t, create);
    OFF(ucg_plan_component_t, destroy); OFF(ucg_plan_component_t, plan);
    OFF(ucg_plan_component_t, prepare); OFF(ucg_plan_component_t, trigger);
    OFF(ucg_plan_component_t, progress); OFF(ucg_plan_component_t, discard);
    OFF(ucg_plan_component_t, print); OFF(ucg_plan_component_t, fault);
    VAL(UCG_PARAM_FIELD_JOB_UID); VAL(UCG_PARAM_FIELD_DATATYPE_CB);
    VAL(UCG_PARAM_FIELD_REDUCE_OP_CB); VAL(UCG_PARAM_FIELD_COMPLETION_CB);
    VAL(UCG_PARAM_FIELD_MPI_IN_PLACE); VAL(UCG_PARAM_FIELD_HANDLE_FAULT);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_SOURCE);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_DESTINATION);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_CONCATENATE);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_BARRIER);
    VAL(UCG_GROUP_COLLECTIVE_MODIFIER_MOCK_EPS);
    VAL(UCG_GROUP_MEMBER_DISTANCE_SELF); VAL(UCG_GROUP_MEMBER_DISTANCE_CACHE);
    VAL(UCG_GROUP_MEMBER_DISTANCE_SOCKET); VAL(UCG_GROUP_MEMBER_DISTANCE_HOST);
    VAL(UCG_GROUP_MEMBER_DISTANCE_NET); VAL(UCG_GROUP_MEMBER_DISTANCE_LAST);
    VAL(UCG_GROUP_PARAM_FIELD_ID); VAL(UCG_GROUP_PARAM_FIELD_DISTANCES);
    VAL(UCG_PLAN_COMPONENT_NAME_MAX);
}

/* ---- the collectives ------------------------------------------------------- */
static int fails;
static unsigned g_rank;
#define CHECK(c, ...) do {                                                      \
        if (!(c)) {                                                             \
            fails++;                                                            \
            fprintf(stderr, "rank %u: FAIL ", g_rank);                          \
            fprintf(stderr, __VA_ARGS__);                                       \
            fputc('\n', stderr);                                                \
        }                                                                       \
    } while (0)

/* MPI_Allreduce / MPI_Reduce parameters as api/ucg_mpi.h's
 * ucg_coll_{allreduce,reduce}_init build them (:53-54, 41-42, 101-120) */
static ucg_collective_params_t make_params(uint16_t mods, uint64_t root, const void *sbuf,
                                           void *rbuf, int count, void *dtype, void *op)
{
    ucg_collective_params_t p;
    memset(&p, 0, sizeof(p));
    UCG_PARAM_TYPE(&p).modifiers = mods;
    UCG_PARAM_TYPE(&p).root      = root;
    p.send.buffer = (void*)sbuf;
    p.send.count  = count;
    p.send.dtype  = dtype;
    p.recv.buffer = rbuf;
    p.recv.count  = count;
    p.recv.dtype  = dtype;
    UCG_PARAM_OP(&p) = op;
    return p;
}

/* member m's input element i: an exact integer */
static double input(unsigned m, int i)
{
    return (double)((int)((m * 7919u + (unsigned)i * 104729u) % 2001u) - 1000);
}

static void fill(void *buf, const mpi_dt_t *d, unsigned m, int n)
{
    int i;
    for (i = 0; i < n; i++) {
        double v = input(m, i);
        if (d->is_float) {
            if (d->size == 4) ((float*)buf)[i] = (float)v; else ((double*)buf)[i] = v;
        } else if (d->size == 4) {
            ((uint32_t*)buf)[i] = (uint32_t)(int32_t)v * 2000000u;   /* wraps when summed */
        } else {
            ((int64_t*)buf)[i] = (int64_t)v;
        }
    }
}

static void expect(void *buf, const mpi_dt_t *d, const mpi_op_t *o, unsigned n_members, int n)
{
    int i;
    unsigned m;
    for (i = 0; i < n; i++) {
        double acc = input(0, i);
        uint32_t acc32 = (uint32_t)(int32_t)input(0, i) * 2000000u;
        for (m = 1; m < n_members; m++) {
            double v = input(m, i);
            uint32_t v32 = (uint32_t)(int32_t)v * 2000000u;
            acc   = o->id == 0 ? acc + v : (v > acc ? v : acc);
            acc32 = o->id == 0 ? acc32 + v32 :
                    ((int32_t)v32 > (int32_t)acc32 ? v32 : acc32);
        }
        if (d->is_float) {
            if (d->size == 4) ((float*)buf)[i] = (float)acc; else ((double*)buf)[i] = acc;
        } else if (d->size == 4) {
            ((uint32_t*)buf)[i] = acc32;
        } else {
            ((int64_t*)buf)[i] = (int64_t)acc;
        }
    }
}

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

/* "latency": BASELINE config 1 through the drop-in boundary - an fp32 SUM
 * allreduce of `count` elements prepared once (the op cache), then `iters`
 * starts, each trigger + progress until the completion callback, as base/
 * runs a persistent MPI_Allreduce; one JSON line from member 0 */
static int latency_run(ucg_group_h grp, unsigned rank, unsigned world, int iters, int count)
{
    const size_t bytes = (size_t)count * 4;
    char *sbuf = malloc(bytes), *rbuf = calloc(1, bytes), *want = malloc(bytes);
    ucg_collective_params_t p;
    ucg_coll_h coll = NULL;
    ucs_status_t st;
    double t0, t1;
    int i, warm = iters / 10 + 1, exact;
    fill(sbuf, &DT_F32, rank, count);
    expect(want, &DT_F32, &OP_SUM, world, count);
    p = make_params(UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                    UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST, 0, sbuf, rbuf, count,
                    &DT_F32, &OP_SUM);
    st = ucg_collective_create(grp, &p, &coll);
    CHECK(st == UCS_OK, "latency: create %d", st);
    if (st != UCS_OK) {
        return 1;
    }
    for (i = 0; i < warm && st == UCS_OK; i++) {
        st = coll_run(grp, coll);
    }
    t0 = now_us();
    for (i = 0; i < iters && st == UCS_OK; i++) {
        st = coll_run(grp, coll);
    }
    t1 = now_us();
    CHECK(st == UCS_OK, "latency: start status %d", st);
    exact = st == UCS_OK && memcmp(rbuf, want, bytes) == 0;
    for (i = 0; !exact && i < count; i++) {
        if (((float*)rbuf)[i] != ((float*)want)[i]) {
            CHECK(0, "latency: result differs at %d: %g, want %g", i, ((float*)rbuf)[i],
                  ((float*)want)[i]);
            break;
        }
    }
    if (rank == 0) {
        printf("{\"config\": \"C1 through ucg_builtin_component: %u-rank allreduce, %d fp32 "
               "SUM, op prepared once, trigger + progress per start\", \"ranks\": %u, "
               "\"bytes\": %zu, \"latency_us\": %.3f, \"iters\": %d, \"bit_exact\": %s}\n",
               world, count, world, bytes, (t1 - t0) / iters, iters, exact ? "true" : "false");
        fflush(stdout);
    }
    coll_destroy(coll);
    free(sbuf);
    free(rbuf);
    free(want);
    return st == UCS_OK && exact ? 0 : 1;
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "host";
    const unsigned rank  = (unsigned)atoi(getenv("RANK") ? getenv("RANK") : "0");
    const unsigned world = (unsigned)atoi(getenv("WORLD_SIZE") ? getenv("WORLD_SIZE") : "1");
    const int device = !strcmp(mode, "device");
    ucg_plan_component_t *comp;
    ucs_config_global_list_entry_t *ce;
    struct ucg_group grp;
    ucg_plan_params_t pp;
    void *config;
    uint8_t am_id = 7;
    unsigned cnt = 0, m, k;
    ucs_status_t st;
    ucg_builtin_dev_ctx_t *dctx = NULL;

    g_rank = rank;
    if (!strcmp(mode, "layout")) {
        dump_layout();
        return 0;
    }
    /* ucg_init: the process-wide parameters (base/ucg_context.c:337-405) */
    memset(&ucg_global_params, 0, sizeof(ucg_global_params));
    ucg_global_params.field_mask = UCG_PARAM_FIELD_JOB_UID | UCG_PARAM_FIELD_DATATYPE_CB |
                                   UCG_PARAM_FIELD_REDUCE_OP_CB |
                                   UCG_PARAM_FIELD_COMPLETION_CB | UCG_PARAM_FIELD_MPI_IN_PLACE;
    ucg_global_params.job_uid = (uint32_t)atoi(getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "1");
    ucg_global_params.datatype.convert             = convert;
    ucg_global_params.datatype.is_integer_f        = is_int;
    ucg_global_params.datatype.is_floating_point_f = is_fp;
    ucg_global_params.reduce_op.reduce_cb_f        = mpi_reduce;
    ucg_global_params.reduce_op.is_sum_f           = is_sum;
    ucg_global_params.reduce_op.is_loc_expected_f  = no_loc;
    ucg_global_params.reduce_op.is_commutative_f   = commutes;
    ucg_global_params.completion.coll_comp_cb_f    = comp_cb;
    ucg_global_params.mpi_in_place                 = &in_place_marker;

    /* ucg_plan_query / ucg_plan_init (base/ucg_plan.c:72-178) */
    comp = find_component("builtin");
    CHECK(comp != NULL, "no \"builtin\" in ucg_plan_components_list");
    if (comp == NULL) {
        return 1;
    }
    k = 0;
    ucs_list_for_each(ce, &ucs_config_global_list, list) {
        k += (ce == &comp->config);
    }
    CHECK(k == 1, "config table not registered");
    CHECK(!strcmp(comp->config.name, "builtin planner") &&
          !strcmp(comp->config.prefix, "BUILTIN_"), "config entry %s/%s",
          comp->config.name, comp->config.prefix);
    st = comp->query(NULL, &cnt);
    CHECK(st == UCS_OK && cnt == 1, "query count %u", cnt);
    st = comp->query(&grp.desc, &cnt);
    CHECK(st == UCS_OK && grp.desc.component == comp && !strcmp(grp.desc.name, "builtin"),
          "query desc");
    config = calloc(1, comp->config.size);
    st = ucs_config_parser_fill_opts(config, comp->config.table, comp->config.prefix);
    CHECK(st == UCS_OK, "config read %d", st);
    grp.pctx = calloc(1, comp->global_ctx_size);
    pp.am_id = &am_id;
    st = comp->init(grp.pctx, &pp, (ucg_plan_config_t*)config);
    CHECK(st == UCS_OK && am_id == 8, "init %d am_id %u", st, am_id);
    if (device) {
        ucg_builtin_dev_ctx_params_t dp;
        memset(&dp, 0, sizeof(dp));
        dp.device = (int)(rank % (unsigned)ucg_builtin_dev_device_count());
        if (ucg_builtin_dev_ctx_create(&dp, &dctx) != UCS_OK) {
            fprintf(stderr, "no device\n");
            return 2;
        }
        ucg_builtin_component_set_classifier(op_cls, dt_cls);
    }

    /* ucg_group_create: member distances of one host */
    memset(grp.cache, 0, sizeof(grp.cache));
    grp.next_coll_id = 0;
    for (m = 0; m < world; m++) {
        grp.distance[m] = m == rank ? UCG_GROUP_MEMBER_DISTANCE_SELF : UCG_GROUP_MEMBER_DISTANCE_HOST;
    }
    memset(&grp.params, 0, sizeof(grp.params));
    grp.params.field_mask   = UCG_GROUP_PARAM_FIELD_ID | UCG_GROUP_PARAM_FIELD_MEMBER_COUNT |
                              UCG_GROUP_PARAM_FIELD_MEMBER_INDEX | UCG_GROUP_PARAM_FIELD_DISTANCES;
    /* COMP_GROUP_ID: the caller's group id (base/ accepts 0, ucg_group.c:302-303) */
    grp.params.id           = getenv("COMP_GROUP_ID") ? (ucg_group_id_t)atoi(getenv("COMP_GROUP_ID")) : 3;
    grp.params.member_count = world;
    grp.params.member_index = rank;
    grp.params.distance     = grp.distance;
    if (posix_memalign(&grp.gctx, 64, comp->per_group_ctx_size) != 0) {
        return 1;
    }
    st = comp->create(grp.pctx, grp.gctx, &grp, &grp.params);
    CHECK(st == UCS_OK, "create %d", st);
    if (st != UCS_OK) {
        return 1;
    }

    if (!strcmp(mode, "latency")) {
        const int rc = latency_run(&grp, rank, world, argc > 2 ? atoi(argv[2]) : 20000,
                                   argc > 3 ? atoi(argv[3]) : 1024);
        comp->destroy(grp.gctx);
        comp->finalize(grp.pctx);
        free(grp.gctx);
        free(grp.pctx);
        free(config);
        return rc;
    }

    {
        /* a group without distances is refused (builtin.c:386-389) */
        ucg_group_params_t bad = grp.params;
        void *g2 = NULL;
        bad.field_mask &= ~(uint64_t)UCG_GROUP_PARAM_FIELD_DISTANCES;
        CHECK(posix_memalign(&g2, 64, comp->per_group_ctx_size) == 0 &&
              comp->create(grp.pctx, g2, &grp, &bad) == UCS_ERR_INVALID_PARAM,
              "create without distances");
        free(g2);
    }

    struct { const char *name; uint16_t mods; int root; mpi_dt_t *dt; mpi_op_t *op; int n;
             int in_place; } cases[] = {
        {"allreduce int32 sum", UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                                UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST, -1, &DT_I32, &OP_SUM, 1000, 0},
        {"allreduce fp64 sum", UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                               UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST, -1, &DT_F64, &OP_SUM, 5000, 0},
        {"allreduce fp32 max in place", UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                                        UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST, -1, &DT_F32, &OP_MAX, 777, 1},
        {"allreduce int64 sum, mock endpoints", UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                                                UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST |
                                                UCG_GROUP_COLLECTIVE_MODIFIER_MOCK_EPS, -1,
         &DT_I64, &OP_SUM, 64, 0},
        {"reduce fp64 sum to the last member", UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                                               UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_DESTINATION,
         (int)world - 1, &DT_F64, &OP_SUM, 3001, 0},
        {"reduce int32 max to member 0", UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE |
                                         UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_DESTINATION,
         0, &DT_I32, &OP_MAX, 100, 0},
    };
    for (k = 0; k < sizeof(cases) / sizeof(cases[0]); k++) {
        const size_t bytes = (size_t)cases[k].n * cases[k].dt->size;
        char *h_send = malloc(bytes), *h_recv = calloc(1, bytes), *want = malloc(bytes);
        void *sbuf = h_send, *rbuf = h_recv;
        const int is_root = cases[k].root < 0 || (unsigned)cases[k].root == rank;
        ucg_coll_h coll = NULL, again = NULL;
        ucg_collective_params_t p;
        int rep;
        fill(h_send, cases[k].dt, rank, cases[k].n);
        if (cases[k].in_place) {
            memcpy(h_recv, h_send, bytes);
        }
        expect(want, cases[k].dt, cases[k].op, world, cases[k].n);
        if (device) {
            sbuf = ucg_builtin_dev_malloc(dctx, bytes);
            rbuf = ucg_builtin_dev_malloc(dctx, bytes);
            ucg_builtin_dev_memcpy(dctx, sbuf, h_send, bytes);
            ucg_builtin_dev_memcpy(dctx, rbuf, h_recv, bytes);
        }
        p = make_params(cases[k].mods, cases[k].root < 0 ? 0 : (uint64_t)cases[k].root,
                        cases[k].in_place ? (void*)&in_place_marker : sbuf,
                        is_root ? rbuf : NULL, cases[k].n, cases[k].dt, cases[k].op);
#ifdef XUCG_REFERENCE_API
        /* the parameters as the reference's own MPI helpers build them
         * (api/ucg_mpi.h:101-120, 156, 162): the same 64 bytes */
        {
            const void *s_arg = cases[k].in_place ? (void*)&in_place_marker : sbuf;
            ucg_coll_h h = NULL;
            if (cases[k].root < 0) {
                st = ucg_coll_allreduce_init(s_arg, rbuf, cases[k].n, cases[k].dt, cases[k].op,
                                             0, cases[k].mods & UCG_GROUP_COLLECTIVE_MODIFIER_MOCK_EPS,
                                             &grp, &h);
            } else {
                st = ucg_coll_reduce_init(s_arg, is_root ? rbuf : NULL, cases[k].n, cases[k].dt,
                                          cases[k].op, (ucg_group_member_index_t)cases[k].root, 0,
                                          &grp, &h);
            }
            CHECK(st == UCS_OK && memcmp(&last_params, &p, sizeof(p)) == 0,
                  "%s: api/ucg_mpi.h builds other parameters (status %d)", cases[k].name, st);
            coll = h;
        }
#else
        st = ucg_collective_create(&grp, &p, &coll);
#endif
        CHECK(st == UCS_OK, "%s: create %d", cases[k].name, st);
        if (st != UCS_OK) {
            continue;
        }
        for (rep = 0; rep < 3; rep++) {
            if (device && rep) {
                ucg_builtin_dev_memcpy(dctx, rbuf, h_recv, bytes);
            }
            st = coll_run(&grp, coll);
            CHECK(st == UCS_OK, "%s: start %d status %d", cases[k].name, rep, st);
            if (st == UCS_OK && is_root) {
                char *got = rbuf;
                if (device) {
                    got = malloc(bytes);
                    ucg_builtin_dev_memcpy(dctx, got, rbuf, bytes);
                }
                CHECK(memcmp(got, want, bytes) == 0, "%s: start %d: result differs",
                      cases[k].name, rep);
                if (device) {
                    free(got);
                }
            }
        }
        if (rank == 0 && k == 0) {
            comp->print(((ucg_op_t*)coll)->plan, &p);
        }
        /* the same parameters again: the cached op (base/ucg_group.c:407-431) */
        coll_destroy(coll);
        st = ucg_collective_create(&grp, &p, &again);
        CHECK(st == UCS_OK && again == coll, "%s: op not reused from the cache", cases[k].name);
        if (st == UCS_OK) {
            st = coll_run(&grp, again);
            CHECK(st == UCS_OK, "%s: cached op status %d", cases[k].name, st);
            coll_destroy(again);
        }
        if (device) {
            ucg_builtin_dev_free(dctx, sbuf);
            ucg_builtin_dev_free(dctx, rbuf);
        }
        free(h_send);
        free(h_recv);
        free(want);
    }

    {
        /* plans without a combine are not this build's: UCS_ERR_UNSUPPORTED
         * (MPI_Bcast, MPI_Allgather, MPI_Alltoall, MPI_Barrier) */
        const uint16_t others[] = {
            UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST | UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_SOURCE,
            UCG_GROUP_COLLECTIVE_MODIFIER_CONCATENATE | UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST,
            0,
            UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE | UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST |
            UCG_GROUP_COLLECTIVE_MODIFIER_BARRIER};
        ucg_collective_type_t t;
        ucg_plan_t *plan;
        for (k = 0; k < sizeof(others) / sizeof(others[0]); k++) {
            t.modifiers = others[k];
            t.root      = 0;
            CHECK(comp->plan(grp.gctx, &t, &plan) == UCS_ERR_UNSUPPORTED,
                  "modifiers 0x%x planned", others[k]);
        }
        CHECK(comp->fault(grp.gctx, 0) == UCS_ERR_NOT_IMPLEMENTED, "fault");
    }

    /* ucg_group_destroy: the component discards its plans and ops */
    comp->destroy(grp.gctx);
    comp->finalize(grp.pctx);
    free(grp.gctx);
    free(grp.pctx);
    free(config);
    if (dctx) {
        ucg_builtin_dev_ctx_destroy(dctx);
    }
    printf("rank %u: %s\n", rank, fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
