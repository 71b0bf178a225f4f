/*
 * builtin_combine.c - host (C) side of the MI355X combine path.
 *
 * Implements include/ucg_builtin_combine.h: the dispatcher that takes the
 * place of ucg_builtin_mpi_reduce() (reference builtin/ops/
 * builtin_comp_step.inl:96-102), the step-scoped device staging used by the
 * REDUCE aggregation branch (:184-232), and the control-path rules (fragment
 * size, recursive-doubling peers) the device path is sized by.
 *
 * The dispatcher never computes a combine itself: it either hands the
 * buffers to the device shim (libucg_builtin_dev.so) or calls the user's
 * reduce_cb_f, exactly as the reference does.
 */
#include "ucg_builtin_combine.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

struct ucg_builtin_combine {
    ucg_builtin_reduce_params_t  params;
    ucg_builtin_combine_config_t cfg;
    ucg_builtin_op_classifier_f  op_cls;
    ucg_builtin_dt_classifier_f  dt_cls;
    ucg_builtin_dev_ctx_t       *dev;        /* NULL: host callback only */
    pthread_mutex_t              lock;       /* AM handler vs async resend */

    /* the step currently staged (or not) */
    struct {
        int              active;   /* a step is open */
        int              on_dev;   /* ... and mirrored on the device */
        void            *op;
        void            *dtype;
        ucg_dev_op_t     dop;
        ucg_dev_dtype_t  ddt;
        char            *recv_buffer;
        size_t           length;
        size_t           dt_len;
    } step;

    uint64_t stats[6];
};

/* ------------------------------------------------------------------------ */
/* configuration                                                            */
/* ------------------------------------------------------------------------ */
/* a size with an optional k/m/g suffix (UCX memunits), dflt when unset or
 * unparsable; shared with the remote-key knobs (builtin_int.h) */
__attribute__((visibility("hidden"))) size_t parse_memunits(const char *s, size_t dflt);
__attribute__((visibility("hidden"))) size_t parse_memunits(const char *s, size_t dflt)
{
    char *end;
    double v;
    if (s == NULL || *s == '\0') {
        return dflt;
    }
    v = strtod(s, &end);
    if (end == s || v < 0) {
        return dflt;
    }
    switch (*end) {
    case 'k': case 'K': v *= 1024.0; break;
    case 'm': case 'M': v *= 1024.0 * 1024.0; break;
    case 'g': case 'G': v *= 1024.0 * 1024.0 * 1024.0; break;
    default: break;
    }
    return (size_t)v;
}

static int parse_bool(const char *s, int dflt)
{
    if (s == NULL || *s == '\0') {
        return dflt;
    }
    if (!strcasecmp(s, "y") || !strcasecmp(s, "yes") || !strcasecmp(s, "on") ||
        !strcmp(s, "1")) {
        return 1;
    }
    if (!strcasecmp(s, "n") || !strcasecmp(s, "no") || !strcasecmp(s, "off") ||
        !strcmp(s, "0")) {
        return 0;
    }
    return dflt;
}

void ucg_builtin_combine_config_read(ucg_builtin_combine_config_t *cfg)
{
    const char *dev = getenv("UCX_BUILTIN_DEV_DEVICE");
    {
        const char *e = getenv("UCX_BUILTIN_DEV_COMBINE");
        cfg->dev_enable = (e && (!strcasecmp(e, "force") || !strcmp(e, "2"))) ? 2 :
                          parse_bool(e, 1);
    }
    cfg->dev_min_bytes = parse_memunits(getenv("UCX_BUILTIN_DEV_MIN_BYTES"),
                                        1u << 20);
    cfg->stage_bytes   = parse_memunits(getenv("UCX_BUILTIN_DEV_STAGE_BYTES"),
                                        16u << 20);
    cfg->stage_slots   = (unsigned)parse_memunits(
                                        getenv("UCX_BUILTIN_DEV_STAGE_SLOTS"), 4);
    cfg->device        = dev ? atoi(dev) : -1;
    {
        /* "0" (and n/no/off/never) turns zero-copy runs off; the field uses
         * the device params' convention (0 = default, NEVER = off) */
        const char *z = getenv("UCX_BUILTIN_DEV_ZCOPY_BYTES");
        if (z && (!strcasecmp(z, "never") || parse_bool(z, 1) == 0)) {
            cfg->zcopy_bytes = UCG_BUILTIN_DEV_ZCOPY_NEVER;
        } else {
            cfg->zcopy_bytes = parse_memunits(z, UCG_BUILTIN_DEV_ZCOPY_DEFAULT);
        }
    }
    {
        /* how a staged step waits for its last launch (ucg_builtin_dev.h) */
        const char *c = getenv("UCX_BUILTIN_DEV_COMPLETION");
        cfg->completion = (c && !strcasecmp(c, "sync")) ? UCG_BUILTIN_DEV_COMPLETION_SYNC :
                                                          UCG_BUILTIN_DEV_COMPLETION_SIGNAL;
    }
    cfg->stream = NULL;
}

/* ------------------------------------------------------------------------ */
/* lifecycle                                                                */
/* ------------------------------------------------------------------------ */
ucs_status_t ucg_builtin_combine_create(const ucg_builtin_reduce_params_t *params,
                                        const ucg_builtin_combine_config_t *cfg,
                                        ucg_builtin_combine_t **cmb_p)
{
    ucg_builtin_combine_t *cmb;
    if (params == NULL || cmb_p == NULL || params->reduce_cb_f == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    cmb = calloc(1, sizeof(*cmb));
    if (cmb == NULL) {
        return UCS_ERR_NO_MEMORY;
    }
    cmb->params = *params;
    if (cfg) {
        cmb->cfg = *cfg;
    } else {
        ucg_builtin_combine_config_read(&cmb->cfg);
    }
    pthread_mutex_init(&cmb->lock, NULL);

    if (cmb->cfg.dev_enable && ucg_builtin_dev_device_count() > 0) {
        ucg_builtin_dev_ctx_params_t dp = {
            .device      = cmb->cfg.device,
            .stream      = cmb->cfg.stream,
            .stage_bytes = cmb->cfg.stage_bytes,
            .stage_slots = cmb->cfg.stage_slots,
            .zcopy_bytes = cmb->cfg.zcopy_bytes,
            .completion  = cmb->cfg.completion
        };
        /* a device that fails to initialise is an error, not a silent
         * downgrade: the caller asked for the device path */
        ucs_status_t st = ucg_builtin_dev_ctx_create(&dp, &cmb->dev);
        if (st != UCS_OK) {
            pthread_mutex_destroy(&cmb->lock);
            free(cmb);
            return st;
        }
    }
    *cmb_p = cmb;
    return UCS_OK;
}

void ucg_builtin_combine_destroy(ucg_builtin_combine_t *cmb)
{
    if (cmb == NULL) {
        return;
    }
    if (cmb->step.active) {
        (void)ucg_builtin_combine_step_end(cmb);
    }
    ucg_builtin_dev_ctx_destroy(cmb->dev);
    pthread_mutex_destroy(&cmb->lock);
    free(cmb);
}

void ucg_builtin_combine_set_classifier(ucg_builtin_combine_t *cmb,
                                        ucg_builtin_op_classifier_f op_cls,
                                        ucg_builtin_dt_classifier_f dt_cls)
{
    cmb->op_cls = op_cls;
    cmb->dt_cls = dt_cls;
}

int ucg_builtin_combine_has_device(ucg_builtin_combine_t *cmb)
{
    return cmb && cmb->dev != NULL;
}

ucg_builtin_dev_ctx_t *ucg_builtin_combine_dev_ctx(ucg_builtin_combine_t *cmb)
{
    return cmb ? cmb->dev : NULL;
}

/* ------------------------------------------------------------------------ */
/* classification                                                           */
/* ------------------------------------------------------------------------ */
/* ucp_datatype_t: class in the low 3 bits (CONTIG = 0), length above
 * (ucp_dt_make_contig / ucp_contig_dt_length, used at builtin/ops/
 * builtin_control.c:1091-1093) */
static size_t contig_dt_length(uintptr_t ucp_dt)
{
    return ((ucp_dt & 7u) == 0) ? (size_t)(ucp_dt >> 3) : 0;
}

static size_t dtype_length(ucg_builtin_combine_t *cmb, void *datatype)
{
    uintptr_t ucp_dt;
    if (datatype == NULL) {
        return 1; /* api/ucg.h:354-356: NULL dtype is a single byte */
    }
    if (cmb->params.convert == NULL) {
        return contig_dt_length((uintptr_t)datatype);
    }
    if (cmb->params.convert(datatype, &ucp_dt) != 0) {
        return 0;
    }
    return contig_dt_length(ucp_dt);
}

size_t ucg_builtin_combine_dtype_length(ucg_builtin_combine_t *cmb, void *datatype)
{
    return cmb ? dtype_length(cmb, datatype) : 0;
}

size_t ucg_builtin_combine_atomic_sum_length(ucg_builtin_combine_t *cmb,
                                             void *reduce_op, void *datatype)
{
    int is_signed = 1;
    size_t len;
    if (cmb == NULL || cmb->params.is_integer_f == NULL ||
        cmb->params.is_sum_f == NULL ||
        !cmb->params.is_integer_f(datatype, &is_signed) || is_signed ||
        !cmb->params.is_sum_f(reduce_op)) {
        return 0;
    }
    len = dtype_length(cmb, datatype);
    return (len == 1 || len == 2 || len == 4 || len == 8) ? len : 0;
}

/* builtin_control.c:872-888: a plan step that reduces needs the reduce_op
 * callbacks, a commutative op (the plans reduce in arrival order) and not
 * MPI_MINLOC/MAXLOC */
ucs_status_t ucg_builtin_combine_check_reduction(ucg_builtin_combine_t *cmb,
                                                 void *reduce_op)
{
    if (cmb == NULL || cmb->params.reduce_cb_f == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (cmb->params.is_commutative_f && !cmb->params.is_commutative_f(reduce_op)) {
        return UCS_ERR_UNSUPPORTED;
    }
    if (cmb->params.is_loc_expected_f && cmb->params.is_loc_expected_f(reduce_op)) {
        return UCS_ERR_UNSUPPORTED;
    }
    return UCS_OK;
}

int ucg_builtin_combine_classify(ucg_builtin_combine_t *cmb, void *reduce_op,
                                 void *datatype, ucg_dev_op_t *op_out,
                                 ucg_dev_dtype_t *dt_out)
{
    int op = -1, dt = -1, is_signed = 0;
    size_t len;

    if (cmb->op_cls) {
        op = cmb->op_cls(reduce_op);
    }
    if (op < 0 && cmb->params.is_sum_f && cmb->params.is_sum_f(reduce_op)) {
        op = UCG_DEV_OP_SUM;
    }
    if (cmb->dt_cls) {
        dt = cmb->dt_cls(datatype);
    }
    if (dt < 0) {
        len = dtype_length(cmb, datatype);
        if (cmb->params.is_integer_f &&
            cmb->params.is_integer_f(datatype, &is_signed)) {
            switch (len) {
            case 1: dt = is_signed ? UCG_DEV_DT_INT8  : UCG_DEV_DT_UINT8;  break;
            case 2: dt = is_signed ? UCG_DEV_DT_INT16 : UCG_DEV_DT_UINT16; break;
            case 4: dt = is_signed ? UCG_DEV_DT_INT32 : UCG_DEV_DT_UINT32; break;
            case 8: dt = is_signed ? UCG_DEV_DT_INT64 : UCG_DEV_DT_UINT64; break;
            default: break;
            }
        } else if (cmb->params.is_floating_point_f &&
                   cmb->params.is_floating_point_f(datatype)) {
            switch (len) {
            case 2: dt = UCG_DEV_DT_FLOAT16; break;
            case 4: dt = UCG_DEV_DT_FLOAT32; break;
            case 8: dt = UCG_DEV_DT_FLOAT64; break;
            default: break;
            }
        }
    }
    if (op < 0 || op >= UCG_DEV_OP_LAST || dt < 0 || dt >= UCG_DEV_DT_LAST ||
        !ucg_builtin_dev_is_supported((ucg_dev_dtype_t)dt, (ucg_dev_op_t)op)) {
        return 0;
    }
    *op_out = (ucg_dev_op_t)op;
    *dt_out = (ucg_dev_dtype_t)dt;
    return 1;
}

/* ------------------------------------------------------------------------ */
/* the combine                                                              */
/* ------------------------------------------------------------------------ */
static ucs_status_t host_reduce(ucg_builtin_combine_t *cmb, void *op, void *src,
                                void *dst, unsigned count, void *dtype,
                                size_t bytes)
{
    int rc = cmb->params.reduce_cb_f(op, (char*)src, (char*)dst, count, dtype);
    cmb->stats[0]++;
    cmb->stats[1] += bytes;
    if (rc != 0) {
        cmb->stats[5]++;
        return UCS_ERR_IO_ERROR;
    }
    return UCS_OK;
}

/* Where a combine runs (measured on MI355X + EPYC 9575F): a
 * device-resident accumulator always on the GPU (the host cannot touch it and
 * nothing crosses PCIe); a host one on reduce_cb_f, because staging moves 3N
 * bytes over PCIe (~22 GiB/s of N) while one host core combines at ~23 GiB/s
 * of N - unless UCX_BUILTIN_DEV_COMBINE=force asks to offload it. */
static int use_device(ucg_builtin_combine_t *cmb, int classified, int dst_on_dev,
                      size_t bytes)
{
    return classified && (dst_on_dev ||
                          (cmb->cfg.dev_enable == 2 && bytes >= cmb->cfg.dev_min_bytes));
}

ucs_status_t ucg_builtin_combine_reduce(ucg_builtin_combine_t *cmb,
                                        void *reduce_op, void *src, void *dst,
                                        int dcount, void *datatype)
{
    ucg_dev_op_t op    = UCG_DEV_OP_SUM;
    ucg_dev_dtype_t dt = UCG_DEV_DT_LAST;   /* set by a successful classify */
    ucs_status_t st;
    size_t bytes;

    if (cmb == NULL || dcount < 0) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (dcount == 0) {
        return UCS_OK;
    }
    pthread_mutex_lock(&cmb->lock);
    if (cmb->dev) {
        int on_dev = ucg_builtin_dev_mem_kind(dst) == UCG_DEV_MEM_DEVICE;
        int cls    = ucg_builtin_combine_classify(cmb, reduce_op, datatype, &op, &dt);
        if (on_dev && !cls) {
            /* reduce_cb_f cannot dereference device memory */
            pthread_mutex_unlock(&cmb->lock);
            return UCS_ERR_UNSUPPORTED;
        }
        bytes = cls ? (size_t)dcount * ucg_builtin_dev_dtype_size(dt) : 0;
        if (use_device(cmb, cls, on_dev, bytes)) {
            st = ucg_builtin_dev_combine_host(cmb->dev, op, dt, dst, src,
                                              (size_t)dcount);
            if (st == UCS_OK) {
                cmb->stats[2]++;
                cmb->stats[3] += bytes;
            }
            pthread_mutex_unlock(&cmb->lock);
            return st;
        }
    }
    st = host_reduce(cmb, reduce_op, src, dst, (unsigned)dcount, datatype,
                     (size_t)dcount * dtype_length(cmb, datatype));
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_step_begin(ucg_builtin_combine_t *cmb,
                                            void *reduce_op, void *datatype,
                                            void *recv_buffer, size_t length)
{
    ucs_status_t st = UCS_OK;
    if (cmb == NULL || (length && recv_buffer == NULL)) {
        return UCS_ERR_INVALID_PARAM;
    }
    pthread_mutex_lock(&cmb->lock);
    if (cmb->step.active) {
        pthread_mutex_unlock(&cmb->lock);
        return UCS_ERR_BUSY;
    }
    memset(&cmb->step, 0, sizeof(cmb->step));
    cmb->step.active      = 1;
    cmb->step.op          = reduce_op;
    cmb->step.dtype       = datatype;
    cmb->step.recv_buffer = (char*)recv_buffer;
    cmb->step.length      = length;
    cmb->step.dt_len      = dtype_length(cmb, datatype);
    if (cmb->step.dt_len == 0) {
        cmb->step.active = 0;
        pthread_mutex_unlock(&cmb->lock);
        return UCS_ERR_INVALID_PARAM;
    }
    if (cmb->dev && length) {
        int on_dev = ucg_builtin_dev_mem_kind(recv_buffer) == UCG_DEV_MEM_DEVICE;
        int cls    = ucg_builtin_combine_classify(cmb, reduce_op, datatype,
                                                  &cmb->step.dop, &cmb->step.ddt);
        if (on_dev && !cls) {
            st = UCS_ERR_UNSUPPORTED;   /* reduce_cb_f cannot touch it */
        } else if (use_device(cmb, cls, on_dev, length)) {
            st = ucg_builtin_dev_stage_begin(cmb->dev, recv_buffer, length);
            if (st == UCS_OK) {
                cmb->step.on_dev = 1;
                cmb->stats[4]++;
            }
        }
        if (st != UCS_OK) {
            cmb->step.active = 0;
        }
    }
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_fragment(ucg_builtin_combine_t *cmb,
                                          size_t offset, const void *src,
                                          size_t length)
{
    ucs_status_t st;
    if (cmb == NULL || !cmb->step.active) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (offset + length > cmb->step.length || length % cmb->step.dt_len) {
        return UCS_ERR_OUT_OF_RANGE;
    }
    pthread_mutex_lock(&cmb->lock);
    if (cmb->step.on_dev) {
        st = ucg_builtin_dev_combine(cmb->dev, cmb->step.dop, cmb->step.ddt,
                                     offset, src, length / cmb->step.dt_len);
        if (st == UCS_OK) {
            cmb->stats[2]++;
            cmb->stats[3] += length;
        }
    } else {
        /* ucg_builtin_mpi_reduce_fragment: count = length / dtype_length */
        st = host_reduce(cmb, cmb->step.op, (void*)src,
                         cmb->step.recv_buffer + offset,
                         (unsigned)(length / cmb->step.dt_len), cmb->step.dtype,
                         length);
    }
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_step_end(ucg_builtin_combine_t *cmb)
{
    ucs_status_t st = UCS_OK;
    if (cmb == NULL || !cmb->step.active) {
        return UCS_ERR_INVALID_PARAM;
    }
    pthread_mutex_lock(&cmb->lock);
    if (cmb->step.on_dev) {
        st = ucg_builtin_dev_stage_end(cmb->dev);
    }
    cmb->step.active = 0;
    cmb->step.on_dev = 0;
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

int ucg_builtin_combine_step_on_device(ucg_builtin_combine_t *cmb)
{
    int on;
    if (cmb == NULL) {
        return 0;
    }
    pthread_mutex_lock(&cmb->lock);
    on = cmb->step.active && cmb->step.on_dev;
    pthread_mutex_unlock(&cmb->lock);
    return on;
}

/* ------------------------------------------------------------------------ */
/* device-resident buffers (the engine's remote-key steps)                  */
/* ------------------------------------------------------------------------ */
static int pool_shareable(void)
{
    const char *e = getenv("UCX_BUILTIN_DEV_POOL_MEM");
    return e != NULL && strcmp(e, "shareable") == 0;
}

void *ucg_builtin_combine_dev_alloc(ucg_builtin_combine_t *cmb, size_t bytes)
{
    void *p;
    if (cmb == NULL || cmb->dev == NULL) {
        return NULL;
    }
    pthread_mutex_lock(&cmb->lock);
    /* exported to the peers. hipMalloc memory (hipIpc keys, checked against
     * the allocation's buffer id) by default: kernels that read peers'
     * imported virtual-memory allocations ran 5-10x longer on one GPU
     * (profiles/r04/r04y: 4 KiB allreduce 95 us against 10 us).
     * UCX_BUILTIN_DEV_POOL_MEM=shareable keeps the pools in shareable
     * allocations (keys that name the physical allocation). */
    p = pool_shareable() ? ucg_builtin_dev_malloc_shareable(cmb->dev, bytes)
                         : ucg_builtin_dev_malloc(cmb->dev, bytes);
    pthread_mutex_unlock(&cmb->lock);
    return p;
}

void ucg_builtin_combine_dev_free(ucg_builtin_combine_t *cmb, void *ptr)
{
    if (cmb == NULL || cmb->dev == NULL || ptr == NULL) {
        return;
    }
    pthread_mutex_lock(&cmb->lock);
    ucg_builtin_dev_free(cmb->dev, ptr);
    pthread_mutex_unlock(&cmb->lock);
}

void ucg_builtin_combine_dev_park(ucg_builtin_combine_t *cmb, void *ptr)
{
    if (cmb == NULL || cmb->dev == NULL || ptr == NULL) {
        return;
    }
    pthread_mutex_lock(&cmb->lock);
    ucg_builtin_dev_park(cmb->dev, ptr);
    pthread_mutex_unlock(&cmb->lock);
}

ucs_status_t ucg_builtin_combine_dev_export(ucg_builtin_combine_t *cmb,
                                            const void *dev_ptr, void *handle)
{
    ucs_status_t st;
    if (cmb == NULL || cmb->dev == NULL) {
        return UCS_ERR_UNSUPPORTED;
    }
    pthread_mutex_lock(&cmb->lock);
    st = ucg_builtin_dev_ipc_export(cmb->dev, dev_ptr, handle);
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_dev_import(ucg_builtin_combine_t *cmb,
                                            const void *handle, void **dev_ptr)
{
    ucs_status_t st;
    if (cmb == NULL || cmb->dev == NULL) {
        return UCS_ERR_UNSUPPORTED;
    }
    pthread_mutex_lock(&cmb->lock);
    st = ucg_builtin_dev_ipc_import(cmb->dev, handle, dev_ptr);
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

void ucg_builtin_combine_dev_release(ucg_builtin_combine_t *cmb, void *dev_ptr)
{
    if (cmb == NULL || cmb->dev == NULL || dev_ptr == NULL) {
        return;
    }
    pthread_mutex_lock(&cmb->lock);
    (void)ucg_builtin_dev_ipc_release(cmb->dev, dev_ptr);
    pthread_mutex_unlock(&cmb->lock);
}

ucs_status_t ucg_builtin_combine_dev_fold(ucg_builtin_combine_t *cmb, void *reduce_op,
                                          void *datatype, void *dst,
                                          const void *const *srcs, unsigned nsrc,
                                          size_t count)
{
    ucg_dev_op_t op;
    ucg_dev_dtype_t dt;
    ucs_status_t st = UCS_OK;
    const void *chunk[16];
    unsigned done = 0;

    if (cmb == NULL || cmb->dev == NULL || srcs == NULL || nsrc == 0) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (!ucg_builtin_combine_classify(cmb, reduce_op, datatype, &op, &dt)) {
        return UCS_ERR_UNSUPPORTED;
    }
    if (count == 0) {
        return UCS_OK;
    }
    pthread_mutex_lock(&cmb->lock);
    /* acc = srcs[0]; acc = srcs[m] (op) acc: k_reduce_tree takes 16
     * operands, the accumulator first, so longer folds continue from dst */
    while (st == UCS_OK && done < nsrc) {
        unsigned n = 0;
        chunk[n++] = done ? dst : srcs[0];
        if (done == 0) {
            done = 1;
        }
        while (n < 16 && done < nsrc) {
            chunk[n++] = srcs[done++];
        }
        st = ucg_builtin_dev_reduce_tree(cmb->dev, op, dt, dst, chunk, n, count);
        cmb->stats[2]++;
        cmb->stats[3] += count * ucg_builtin_dev_dtype_size(dt) * (n - 1);
    }
    if (st == UCS_OK) {
        st = ucg_builtin_dev_complete(cmb->dev);   /* before READY / DONE go out */
    }
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_dev_copy(ucg_builtin_combine_t *cmb, void *dst,
                                          const void *src, size_t bytes)
{
    ucs_status_t st;
    void *const d[1]       = {dst};
    const void *const s[1] = {src};
    if (cmb == NULL || cmb->dev == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (bytes == 0 || dst == src) {
        return UCS_OK;
    }
    pthread_mutex_lock(&cmb->lock);
    st = ucg_builtin_dev_copy_multi(cmb->dev, d, s, 1, bytes);
    if (st == UCS_OK) {
        st = ucg_builtin_dev_complete(cmb->dev);   /* before READY / DONE go out */
    }
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_dev_copy_n(ucg_builtin_combine_t *cmb,
                                            void *const *dsts, const void *const *srcs,
                                            unsigned n, size_t bytes)
{
    ucs_status_t st;
    if (cmb == NULL || cmb->dev == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (bytes == 0 || n == 0) {
        return UCS_OK;
    }
    pthread_mutex_lock(&cmb->lock);
    st = ucg_builtin_dev_copy_multi(cmb->dev, dsts, srcs, n, bytes);
    if (st == UCS_OK) {
        st = ucg_builtin_dev_complete(cmb->dev);
    }
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_dev_butterfly(ucg_builtin_combine_t *cmb, void *reduce_op,
                                               void *datatype, void *dst,
                                               const void *const *srcs, unsigned nsrc,
                                               unsigned self, size_t count)
{
    ucg_dev_op_t op;
    ucg_dev_dtype_t dt;
    ucs_status_t st;
    if (cmb == NULL || cmb->dev == NULL) {
        return UCS_ERR_INVALID_PARAM;
    }
    if (!ucg_builtin_combine_classify(cmb, reduce_op, datatype, &op, &dt)) {
        return UCS_ERR_UNSUPPORTED;
    }
    if (count == 0) {
        return UCS_OK;
    }
    pthread_mutex_lock(&cmb->lock);
    st = ucg_builtin_dev_reduce_multi(cmb->dev, op, dt, dst, srcs, nsrc, self, count);
    if (st == UCS_OK) {
        cmb->stats[2]++;
        cmb->stats[3] += count * ucg_builtin_dev_dtype_size(dt) * nsrc;
        st = ucg_builtin_dev_complete(cmb->dev);
    }
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

ucs_status_t ucg_builtin_combine_mem_reg(ucg_builtin_combine_t *cmb, void *ptr, size_t bytes)
{
    ucs_status_t st;
    if (cmb == NULL || cmb->dev == NULL) {
        return UCS_ERR_UNSUPPORTED;
    }
    pthread_mutex_lock(&cmb->lock);
    st = ucg_builtin_dev_host_register(cmb->dev, ptr, bytes);
    pthread_mutex_unlock(&cmb->lock);
    return st;
}

void ucg_builtin_combine_mem_dereg(ucg_builtin_combine_t *cmb, void *ptr)
{
    if (cmb == NULL || cmb->dev == NULL || ptr == NULL) {
        return;
    }
    pthread_mutex_lock(&cmb->lock);
    (void)ucg_builtin_dev_host_unregister(cmb->dev, ptr);
    pthread_mutex_unlock(&cmb->lock);
}

void ucg_builtin_combine_stats(ucg_builtin_combine_t *cmb, uint64_t out[6])
{
    int i;
    for (i = 0; i < 6; i++) {
        out[i] = cmb ? cmb->stats[i] : 0;
    }
}

/* ------------------------------------------------------------------------ */
/* control-path rules                                                       */
/* ------------------------------------------------------------------------ */
size_t ucg_builtin_step_fragment_length(size_t max_short, size_t dt_len)
{
    /* max_short minus the 8-byte ucg_builtin_header_t, rounded down to a
     * whole element (builtin_control.c:434 and :462) */
    size_t m;
    if (dt_len == 0 || max_short <= 8) {
        return 0;
    }
    m = max_short - 8;
    return m - (m % dt_len);
}

uint64_t ucg_builtin_step_fragments_total(size_t length, size_t frag_len,
                                          unsigned ep_cnt)
{
    if (frag_len == 0) {
        return 0;
    }
    return (uint64_t)ep_cnt * (length / frag_len + ((length % frag_len) > 0));
}

size_t ucg_builtin_dev_chunk_bytes(size_t length, size_t frag_len,
                                   size_t slot_bytes)
{
    size_t per;
    if (frag_len == 0 || slot_bytes < frag_len) {
        return frag_len;
    }
    /* whole fragments per ring slot, never more than the step itself */
    per = (slot_bytes / frag_len) * frag_len;
    return per < length ? per : length;
}

unsigned ucg_builtin_recursive_steps(uint64_t count, unsigned factor)
{
    uint64_t step_size = 1;
    unsigned steps = 0;
    if (factor < 2 || count == 0) {
        return 0;
    }
    while (step_size < count) {
        step_size *= factor;
        steps++;
    }
    return (step_size == count) ? steps : 0;
}

uint64_t ucg_builtin_recursive_peer(uint64_t my, unsigned step,
                                    unsigned factor, unsigned peer_idx)
{
    uint64_t step_size = 1, base;
    unsigned i;
    for (i = 1; i < step; i++) {
        step_size *= factor;
    }
    base = my - (my % (step_size * factor));
    return base + ((my - base + step_size * peer_idx) % (step_size * factor));
}
