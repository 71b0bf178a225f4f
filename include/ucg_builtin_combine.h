/*
 * ucg_builtin_combine.h - host (C) side of the MI355X combine path inside
 * UCG's builtin planner.
 *
 * This is what builtin/ops and builtin/plan call instead of invoking
 * reduce_cb_f directly. It decides, per call, whether the combine runs on
 * the device (through include/ucg_builtin_dev.h) or through the user's
 * reduce_cb_f on the host, and restates the control-path rules the device
 * path depends on. Reference anchors (paths relative to the reference tree):
 *
 *   ucg_builtin_combine_reduce()      replaces the body of
 *                                     ucg_builtin_mpi_reduce(),
 *                                     builtin/ops/builtin_comp_step.inl:96-102
 *   ucg_builtin_combine_step_begin/
 *   ucg_builtin_combine_fragment/
 *   ucg_builtin_combine_step_end()    the REDUCE aggregation branch of
 *                                     ucg_builtin_step_recv_handle_chunk(),
 *                                     :184-232, around a whole step (begin at
 *                                     ucg_builtin_step_execute, builtin/ops/
 *                                     builtin_data.c:584; end before the next
 *                                     step's send, builtin_comp_step.inl:60-95,
 *                                     or completion, :8-38)
 *   ucg_builtin_combine_create/
 *   ucg_builtin_combine_destroy()     per-group state created in
 *                                     ucg_builtin_create(), builtin/builtin.c:
 *                                     376-456, freed in ucg_builtin_destroy()
 *   ucg_builtin_step_fragment_length/
 *   ucg_builtin_step_fragments_total() builtin/ops/builtin_control.c:434,462-465
 *   ucg_builtin_recursive_*()         builtin/plan/builtin_recursive.c:20-228
 *
 * The callback types mirror ucg_params_t.datatype and .reduce_op
 * (api/ucg.h:129-160) exactly; ucp_datatype_t is carried as uintptr_t.
 */
#ifndef UCG_BUILTIN_COMBINE_H_
#define UCG_BUILTIN_COMBINE_H_

#include "ucg_builtin_dev.h"

#ifdef __cplusplus
extern "C" {
#endif

/* api/ucg.h:129-160 (ucg_params_t.datatype / .reduce_op) */
typedef struct ucg_builtin_reduce_params {
    int (*reduce_cb_f)(void *reduce_op, char *src, char *dst, unsigned count,
                       void *datatype);
    int (*is_sum_f)(void *reduce_op);
    int (*is_loc_expected_f)(void *reduce_op);
    int (*is_commutative_f)(void *reduce_op);
    int (*convert)(void *datatype, uintptr_t *ucp_datatype);
    int (*is_integer_f)(void *datatype, int *is_signed);
    int (*is_floating_point_f)(void *datatype);
} ucg_builtin_reduce_params_t;

/* Builtin-private knobs, read from the environment with the builtin
 * planner's prefix (UCX_BUILTIN_, builtin/builtin.c:1015). */
typedef struct ucg_builtin_combine_config {
    int      dev_enable;     /* UCX_BUILTIN_DEV_COMBINE n|y|force (0/1/2, y):
                                y: device-resident buffers on the GPU, host
                                buffers on reduce_cb_f; force: host buffers
                                of >= dev_min_bytes are staged on the GPU too */
    size_t   dev_min_bytes;  /* UCX_BUILTIN_DEV_MIN_BYTES    (default 1 MiB)   */
    size_t   stage_bytes;    /* UCX_BUILTIN_DEV_STAGE_BYTES  (default 16 MiB)  */
    unsigned stage_slots;    /* UCX_BUILTIN_DEV_STAGE_SLOTS  (default 4)       */
    int      device;         /* UCX_BUILTIN_DEV_DEVICE       (default -1)      */
    size_t   zcopy_bytes;    /* UCX_BUILTIN_DEV_ZCOPY_BYTES  (default 64k;
                                0, n, never: UCG_BUILTIN_DEV_ZCOPY_NEVER)      */
    int      completion;     /* UCX_BUILTIN_DEV_COMPLETION   signal|sync (default
                                signal: UCG_BUILTIN_DEV_COMPLETION_*)          */
    void    *stream;         /* the caller's HIP stream (hipStream_t), or NULL:
                                the device work of this combine - kernels over
                                the caller's device buffers included - is then
                                queued behind the caller's own work on it, so
                                buffers produced asynchronously there are read
                                only once written. NULL = a private stream
                                (the caller must then complete its work on the
                                buffers before starting an op). Not read from
                                the environment. */
} ucg_builtin_combine_config_t;

typedef struct ucg_builtin_combine ucg_builtin_combine_t;

/* builtin-private classifier (not part of api/): maps the opaque MPI handles
 * to the device enums; return -1 when unknown. Without it only SUM (via
 * is_sum_f) and size/int/float-classified types are device-eligible, and a
 * 2-byte float is taken as fp16 (api/ cannot tell fp16 from bf16). */
typedef int (*ucg_builtin_op_classifier_f)(void *reduce_op);
typedef int (*ucg_builtin_dt_classifier_f)(void *datatype);

void         ucg_builtin_combine_config_read(ucg_builtin_combine_config_t *cfg);
ucs_status_t ucg_builtin_combine_create(const ucg_builtin_reduce_params_t *params,
                                        const ucg_builtin_combine_config_t *cfg,
                                        ucg_builtin_combine_t **cmb_p);
void         ucg_builtin_combine_destroy(ucg_builtin_combine_t *cmb);
void         ucg_builtin_combine_set_classifier(ucg_builtin_combine_t *cmb,
                                                ucg_builtin_op_classifier_f op_cls,
                                                ucg_builtin_dt_classifier_f dt_cls);
/* 1 when (op, dtype) can run on the device; fills the enums. */
int          ucg_builtin_combine_classify(ucg_builtin_combine_t *cmb,
                                          void *reduce_op, void *datatype,
                                          ucg_dev_op_t *op, ucg_dev_dtype_t *dt);
/* Contiguous element length of an opaque datatype (datatype.convert +
 * ucp_contig_dt_length, builtin/ops/builtin_control.c:1091-1093); 0 if not
 * contiguous. NULL is one byte (api/ucg.h:354-356). */
size_t       ucg_builtin_combine_dtype_length(ucg_builtin_combine_t *cmb,
                                              void *datatype);
/* 1 when a device context is attached (a GPU was found and enabled). */
int          ucg_builtin_combine_has_device(ucg_builtin_combine_t *cmb);
ucg_builtin_dev_ctx_t *ucg_builtin_combine_dev_ctx(ucg_builtin_combine_t *cmb);

/* The combine itself: dst[i] = src[i] (op) dst[i] on host memory, the exact
 * contract of reduce_cb_f. Whole-buffer calls of at least dev_min_bytes go
 * to the device (H2D -> kernel -> D2H); everything else, and every op or
 * type the device cannot classify, calls reduce_cb_f. The callback's return
 * value is propagated here (the reference discards it). */
/* The atomic-packer condition of ucg_builtin_step_select_packers
 * (builtin/ops/builtin_control.c:535-575): an unsigned integer datatype and
 * is_sum_f(op). Returns the element length (1, 2, 4 or 8), else 0. */
size_t       ucg_builtin_combine_atomic_sum_length(ucg_builtin_combine_t *cmb,
                                                   void *reduce_op,
                                                   void *datatype);

/* The checks ucg_builtin_step_create makes for a step that reduces
 * (builtin/ops/builtin_control.c:872-888): UCS_ERR_UNSUPPORTED for a
 * non-commutative op (is_commutative_f) or MPI_MINLOC/MAXLOC
 * (is_loc_expected_f). */
ucs_status_t ucg_builtin_combine_check_reduction(ucg_builtin_combine_t *cmb,
                                                 void *reduce_op);

ucs_status_t ucg_builtin_combine_reduce(ucg_builtin_combine_t *cmb,
                                        void *reduce_op, void *src, void *dst,
                                        int dcount, void *datatype);

/* Step-scoped device staging for fragmented REDUCE steps: between begin and
 * end the step's receive buffer is mirrored on the device, every fragment is
 * copied into the pinned ring before the call returns and consecutive ones
 * are combined in one launch. Steps below dev_min_bytes, or not classified,
 * fall back to reduce_cb_f per fragment with identical results. */
ucs_status_t ucg_builtin_combine_step_begin(ucg_builtin_combine_t *cmb,
                                            void *reduce_op, void *datatype,
                                            void *recv_buffer, size_t length);
ucs_status_t ucg_builtin_combine_fragment(ucg_builtin_combine_t *cmb,
                                          size_t offset, const void *src,
                                          size_t length);
ucs_status_t ucg_builtin_combine_step_end(ucg_builtin_combine_t *cmb);
/* 1 when the open step is mirrored on the device (its fragments land in the
 * accumulator only at step_end), 0 when each fragment is combined into the
 * recv buffer by the time ucg_builtin_combine_fragment returns. */
int          ucg_builtin_combine_step_on_device(ucg_builtin_combine_t *cmb);

/* ---- device-resident buffers: the engine's remote-key steps ------------- */
/* The zero-copy form of a step (the reference's rkey exchange and
 * SEND_GET_ZCOPY, builtin_control.c:1014-1076, builtin_data.c:326-340) for
 * buffers in GPU memory: each member exposes a device buffer of its own
 * through a HIP IPC handle (the packed remote key, once per op), and a
 * receiver reads its peers' buffers over xGMI in one kernel. Every call takes
 * the combine's lock and returns once the device work is complete. */
void        *ucg_builtin_combine_dev_alloc(ucg_builtin_combine_t *cmb, size_t bytes);
void         ucg_builtin_combine_dev_free(ucg_builtin_combine_t *cmb, void *ptr);
/* keep an exported buffer a peer may still read: keys retired, memory never
 * reused (ucg_builtin_dev_park) */
void         ucg_builtin_combine_dev_park(ucg_builtin_combine_t *cmb, void *ptr);
ucs_status_t ucg_builtin_combine_dev_export(ucg_builtin_combine_t *cmb,
                                            const void *dev_ptr, void *handle);
ucs_status_t ucg_builtin_combine_dev_import(ucg_builtin_combine_t *cmb,
                                            const void *handle, void **dev_ptr);
void         ucg_builtin_combine_dev_release(ucg_builtin_combine_t *cmb, void *dev_ptr);
/* dst = srcs[nsrc-1] (op) (... (srcs[1] (op) srcs[0])): the accumulator
 * srcs[0] with every peer's data reduced into it in the given (arrival)
 * order, as reduce_cb_f would one message at a time (builtin_comp_step.inl:
 * 213-221). Any nsrc >= 1 (launched 16 operands at a time); dst may alias
 * srcs[0]; srcs may be peer-mapped. UCS_ERR_UNSUPPORTED for an (op, dtype)
 * the device cannot classify. */
ucs_status_t ucg_builtin_combine_dev_fold(ucg_builtin_combine_t *cmb, void *reduce_op,
                                          void *datatype, void *dst,
                                          const void *const *srcs, unsigned nsrc,
                                          size_t count);
/* dst[0:bytes] = src[0:bytes], either side device or peer-mapped memory */
ucs_status_t ucg_builtin_combine_dev_copy(ucg_builtin_combine_t *cmb, void *dst,
                                          const void *src, size_t bytes);
/* n copies of `bytes` each in one launch (ucg_builtin_dev_copy_multi), n <= 16 */
ucs_status_t ucg_builtin_combine_dev_copy_n(ucg_builtin_combine_t *cmb,
                                            void *const *dsts, const void *const *srcs,
                                            unsigned n, size_t bytes);
/* dst = V(self, log2 nsrc) of the recursive-doubling association over the
 * nsrc operands (ucg_builtin_dev_reduce_multi): the result member `self`
 * holds after the reference's recursive doubling, in one pass */
ucs_status_t ucg_builtin_combine_dev_butterfly(ucg_builtin_combine_t *cmb, void *reduce_op,
                                               void *datatype, void *dst,
                                               const void *const *srcs, unsigned nsrc,
                                               unsigned self, size_t count);

/* The memory registration of a persistent op's host recv buffer (the
 * reference registers an op's buffers after MEM_REG_OPT_CNT starts,
 * builtin_control.c:276-286, 345-373; dropped in discard, :1289-1292): a
 * staged step's H2D / D2H of a registered buffer moves by DMA, with no staging
 * copy in the runtime. UCS_ERR_UNSUPPORTED without a device. */
ucs_status_t ucg_builtin_combine_mem_reg(ucg_builtin_combine_t *cmb, void *ptr,
                                         size_t bytes);
void         ucg_builtin_combine_mem_dereg(ucg_builtin_combine_t *cmb, void *ptr);

/* [0] host calls, [1] host bytes, [2] device calls, [3] device bytes,
 * [4] steps staged on the device, [5] callback errors seen */
void         ucg_builtin_combine_stats(ucg_builtin_combine_t *cmb,
                                       uint64_t out[6]);

/* ---- control-path rules the device path depends on ---------------------- */
/* builtin/ops/builtin_control.c:434,462: whole-element AM-short fragment */
size_t       ucg_builtin_step_fragment_length(size_t max_short, size_t dt_len);
/* builtin/ops/builtin_control.c:463-465 */
uint64_t     ucg_builtin_step_fragments_total(size_t length, size_t frag_len,
                                              unsigned ep_cnt);
/* Device launch granularity for a fragmented step: fragments are aggregated
 * into runs of at most this many bytes (a whole number of fragments). */
size_t       ucg_builtin_dev_chunk_bytes(size_t length, size_t frag_len,
                                         size_t slot_bytes);
/* builtin/plan/builtin_recursive.c:76-88: number of recursive steps for
 * `count` members and `factor`, or 0 when count is not a power of factor */
unsigned     ucg_builtin_recursive_steps(uint64_t count, unsigned factor);
/* builtin/plan/builtin_recursive.c:158-169: peer #peer_idx (1..factor-1) of
 * member `my` at 1-based step `step` */
uint64_t     ucg_builtin_recursive_peer(uint64_t my, unsigned step,
                                        unsigned factor, unsigned peer_idx);

#ifdef __cplusplus
}
#endif

#endif
