/*
 * ucg_builtin_dev.h - C-ABI of the MI355X device combine behind UCG's builtin
 * planner (the "device shim").
 *
 * This header is the drop-in boundary for ONE path of openucx/xucg: the local
 * element-wise reduce/combine `dst[i] = src[i] (op) dst[i]` that builtin/ops
 * applies to every incoming fragment of a reduce/allreduce step.
 *
 * Reference interfaces each entry point replaces or serves (paths relative to
 * the reference tree):
 *
 *   ucg_builtin_dev_reduce()        <- ucg_builtin_mpi_reduce()
 *                                      builtin/ops/builtin_comp_step.inl:96-102,
 *                                      i.e. the reduce_cb_f contract
 *                                      api/ucg.h:149-150, for buffers that are
 *                                      already device-resident.
 *   ucg_builtin_dev_combine_host()  <- ucg_builtin_mpi_reduce_single()
 *                                      builtin/ops/builtin_comp_step.inl:104-110
 *                                      (one whole-buffer call on host memory,
 *                                      H2D -> kernel -> D2H, pipelined).
 *   ucg_builtin_dev_stage_begin/
 *   ucg_builtin_dev_combine/
 *   ucg_builtin_dev_stage_end()     <- ucg_builtin_mpi_reduce_fragment()
 *                                      builtin/ops/builtin_comp_step.inl:112-120
 *                                      called per fragment from
 *                                      ucg_builtin_step_recv_handle_chunk()
 *                                      :184-232; src is borrowed (released at
 *                                      :443-449) so it is copied into a pinned
 *                                      ring before the call returns.
 *   ucg_builtin_dev_reduce_multi()  <- the per-element association that the
 *                                      recursive-doubling plan produces over
 *                                      2^k ranks (builtin/plan/
 *                                      builtin_recursive.c:158-169), evaluated
 *                                      in one pass (one-shot reduce-scatter).
 *   ucg_builtin_dev_reduce_tree()   <- the same for the tree plan's fan-in at
 *                                      its root (builtin/plan/builtin_tree.c:
 *                                      262-380, builtin_comp_step.inl:213-221),
 *                                      any group size.
 *   ucg_builtin_dev_ctx_create/
 *   ucg_builtin_dev_ctx_destroy()   <- per-group state that lives in
 *                                      struct ucg_builtin_group_ctx
 *                                      builtin/builtin.c:66-90, created and
 *                                      destroyed by ucg_builtin_create/destroy
 *                                      :376-524.
 *
 * Semantics (the oracle in oracle/combine_ref.c restates them on the CPU and
 * tests/golden pins them against MPICH 3.3.2 MPI_Reduce_local):
 *   - dst is the in/out accumulator, src the incoming operand, count elements.
 *   - SUM/PROD on integers wrap modulo 2^n; on floats they are one IEEE-754
 *     round-to-nearest-even op, subnormals preserved, and NaN results follow
 *     the x86-SSE rule of the host MPI library: a NaN dst is returned quieted,
 *     else a NaN src is returned quieted, else an invalid op gives the default
 *     NaN (sign set, quiet bit set).
 *   - MAX is dst = (dst > src) ? dst : src, MIN is dst = (dst < src) ? dst :
 *     src (so NaN and signed-zero behaviour is that of the C ternary).
 *   - fp16 / bf16 compute in fp32 and round once (RNE) to the storage type.
 *   - LAND/LOR/LXOR/BAND/BOR/BXOR are defined for integer types only.
 *
 * All entry points are plain C: pointers, sizes, enums. No HIP or torch types
 * appear in a signature; a HIP stream is passed as `void *`.
 */
#ifndef UCG_BUILTIN_DEV_H_
#define UCG_BUILTIN_DEV_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/*
 * Status codes. Inside a UCX build define UCG_BUILTIN_DEV_HAVE_UCS and include
 * <ucs/type/status.h> first; the values below are UCX's own (ucs_status_t).
 */
#ifdef UCG_BUILTIN_DEV_HAVE_UCS
#include <ucs/type/status.h>
#else
#ifndef UCG_BUILTIN_DEV_UCS_STATUS_DEFINED
#define UCG_BUILTIN_DEV_UCS_STATUS_DEFINED
typedef enum {
    UCS_OK                  =   0,
    UCS_INPROGRESS          =   1,
    UCS_ERR_NO_RESOURCE     =  -2,
    UCS_ERR_IO_ERROR        =  -3,
    UCS_ERR_NO_MEMORY       =  -4,
    UCS_ERR_INVALID_PARAM   =  -5,
    UCS_ERR_NOT_IMPLEMENTED =  -8,
    UCS_ERR_NO_DEVICE       = -14,
    UCS_ERR_BUSY            = -15,
    UCS_ERR_CANCELED        = -16,
    UCS_ERR_OUT_OF_RANGE    = -19,
    UCS_ERR_TIMED_OUT       = -20,
    UCS_ERR_EXCEEDS_LIMIT   = -21,
    UCS_ERR_UNSUPPORTED     = -22,
    UCS_ERR_CONNECTION_RESET = -25
} ucs_status_t;
#endif
#endif

/* Element types the device path can classify (see ucg_builtin_combine.h for
 * the mapping from the opaque MPI datatype of api/ucg.h:131-137). */
typedef enum ucg_dev_dtype {
    UCG_DEV_DT_INT8 = 0,
    UCG_DEV_DT_UINT8,
    UCG_DEV_DT_INT16,
    UCG_DEV_DT_UINT16,
    UCG_DEV_DT_INT32,
    UCG_DEV_DT_UINT32,
    UCG_DEV_DT_INT64,
    UCG_DEV_DT_UINT64,
    UCG_DEV_DT_FLOAT16,
    UCG_DEV_DT_BFLOAT16,
    UCG_DEV_DT_FLOAT32,
    UCG_DEV_DT_FLOAT64,
    UCG_DEV_DT_LAST
} ucg_dev_dtype_t;

/* Reduction operators (MPI predefined ops without MINLOC/MAXLOC, which the
 * reference rejects: builtin/ops/builtin_control.c:884-887). */
typedef enum ucg_dev_op {
    UCG_DEV_OP_SUM = 0,
    UCG_DEV_OP_PROD,
    UCG_DEV_OP_MAX,
    UCG_DEV_OP_MIN,
    UCG_DEV_OP_LAND,
    UCG_DEV_OP_LOR,
    UCG_DEV_OP_LXOR,
    UCG_DEV_OP_BAND,
    UCG_DEV_OP_BOR,
    UCG_DEV_OP_BXOR,
    UCG_DEV_OP_LAST
} ucg_dev_op_t;

/* Synthetic input distributions. */
typedef enum ucg_dev_dist {
    UCG_DEV_DIST_EXACT = 0, /* integers uniform in [-1024, 1024], cast */
    UCG_DEV_DIST_ROUND,     /* random mantissa x 2^U[-8,8], random sign;
                               integer types: full-range random bits */
    UCG_DEV_DIST_SPECIAL,   /* the fixed special-value table, hashed index */
    UCG_DEV_DIST_LAST
} ucg_dev_dist_t;

typedef struct ucg_builtin_dev_ctx ucg_builtin_dev_ctx_t;

typedef struct ucg_builtin_dev_ctx_params {
    int      device;       /* HIP device ordinal; -1 = the calling thread's */
    void    *stream;       /* hipStream_t to launch on; NULL = create one
                              (so the legacy null stream cannot be chosen) */
    size_t   stage_bytes;  /* pinned staging slot size; 0 = 16 MiB */
    unsigned stage_slots;  /* staging ring depth; 0 = 4 */
    size_t   zcopy_bytes;  /* staged runs of at most this many bytes are read
                              by the kernel from the pinned slot over PCIe,
                              with no H2D copy; 0 = 64 KiB,
                              UCG_BUILTIN_DEV_ZCOPY_NEVER = always copy */
    int      completion;   /* how stage_end waits for the step's last launch
                              (UCG_BUILTIN_DEV_COMPLETION_*; 0 = SIGNAL) */
} ucg_builtin_dev_ctx_params_t;

#define UCG_BUILTIN_DEV_ZCOPY_DEFAULT ((size_t)64 << 10)
#define UCG_BUILTIN_DEV_ZCOPY_NEVER   ((size_t)-1)

/* Completion wait of a staged step (ucg_builtin_dev_stage_end) whose result
 * is in device memory or pinned host memory:
 *   SIGNAL  a one-workgroup kernel queued behind the step publishes a sequence
 *           number to a pinned host word with a system-scope release store;
 *           the host spins on it (then blocks in hipStreamSynchronize if the
 *           step runs longer than 200 us). 8.8-9.7 us per small step against
 *           11.5-11.8 us (tools/tune_latency, profiles/r02/r02d).
 *   SYNC    hipStreamSynchronize.
 * A result copied back into pageable host memory always takes SYNC. */
#define UCG_BUILTIN_DEV_COMPLETION_SIGNAL 1
#define UCG_BUILTIN_DEV_COMPLETION_SYNC   2

/* ---- introspection (no GPU needed) ---------------------------------------*/
size_t      ucg_builtin_dev_dtype_size(ucg_dev_dtype_t dt);
int         ucg_builtin_dev_is_supported(ucg_dev_dtype_t dt, ucg_dev_op_t op);
const char *ucg_builtin_dev_version(void);
/* Thread-local text of the last error reported by this library. */
const char *ucg_builtin_dev_last_error(void);
/* Number of HIP devices visible (0 when none); never initialises a context. */
int         ucg_builtin_dev_device_count(void);

/* Where a buffer lives (hipPointerGetAttributes): the dispatcher keeps host
 * buffers on the host CPU by default and sends device-resident ones (a
 * GPU-aware MPI's recv buffer, an IPC-mapped peer) to the GPU. */
enum {
    UCG_DEV_MEM_HOST   = 0,   /* host memory unknown to HIP (pageable)    */
    UCG_DEV_MEM_PINNED = 1,   /* host memory registered with / from HIP   */
    UCG_DEV_MEM_DEVICE = 2    /* GPU memory (local, peer-mapped, managed) */
};
int         ucg_builtin_dev_mem_kind(const void *ptr);

/* ---- per-group device context --------------------------------------------*/
ucs_status_t ucg_builtin_dev_ctx_create(const ucg_builtin_dev_ctx_params_t *params,
                                        ucg_builtin_dev_ctx_t **ctx_p);
void         ucg_builtin_dev_ctx_destroy(ucg_builtin_dev_ctx_t *ctx);
void        *ucg_builtin_dev_ctx_stream(ucg_builtin_dev_ctx_t *ctx);
/* Wait for all work queued on the context's stream(s). */
ucs_status_t ucg_builtin_dev_sync(ucg_builtin_dev_ctx_t *ctx);
/* Wait for the work queued on the context's launch stream the way the
 * context ends a staged step (params.completion): with the completion word a
 * one-workgroup kernel behind the work writes, spun on for 200 us before the
 * runtime's blocking wait; with COMPLETION_SYNC, hipStreamSynchronize. */
ucs_status_t ucg_builtin_dev_complete(ucg_builtin_dev_ctx_t *ctx);

/* ---- device-resident combine ---------------------------------------------*/
/* dst[i] = src[i] (op) dst[i] for i < count; dst/src are device pointers.
 * Asynchronous on the context stream. dst == src is allowed (self-combine);
 * partially overlapping ranges are not. */
ucs_status_t ucg_builtin_dev_reduce(ucg_builtin_dev_ctx_t *ctx, ucg_dev_op_t op,
                                    ucg_dev_dtype_t dt, void *dst,
                                    const void *src, size_t count);

/* The all-gather half of a one-shot reduce-scatter + all-gather (SURVEY.md
 * 8e): dst[r * shard_bytes + i] = srcs[r][i] for r < nsrc, every source read in
 * one launch (srcs may be peer-mapped device pointers: member r's shard over
 * xGMI). A NULL source leaves its row of dst untouched (a member's own shard,
 * already in place), so the other N-1 rows still go in one launch with every
 * link streaming. A plain copy; no reference counterpart (the reference has
 * no all-gather of reduced shards). nsrc <= 16, at least one source non-NULL. */
ucs_status_t ucg_builtin_dev_gather_multi(ucg_builtin_dev_ctx_t *ctx, void *dst,
                                          const void *const *srcs, unsigned nsrc,
                                          size_t shard_bytes);

/* n independent copies of nbytes each in one launch: dsts[i][0:nbytes] =
 * srcs[i][0:nbytes]. Either side may be peer-mapped (a push over xGMI when the
 * destinations are peers' buffers); workgroups are dealt round-robin over the
 * pairs so every link streams at once. Sources may repeat (a broadcast of one
 * shard to every peer); destinations must not overlap. n <= 16. */
ucs_status_t ucg_builtin_dev_copy_multi(ucg_builtin_dev_ctx_t *ctx,
                                        void *const *dsts, const void *const *srcs,
                                        unsigned n, size_t nbytes);

/* One-shot multi-operand combine in the recursive-doubling association of
 * builtin/plan/builtin_recursive.c:158-169 as seen from member `self`:
 *   V(r,0) = srcs[r];  V(r,k) = V(r ^ 2^(k-1), k-1) (op) V(r, k-1)
 * (left operand = src, right = dst of the reduce_cb_f contract), and writes
 * dst[i] = V(self, log2(nsrc))[i]. nsrc must be a power of two <= 16; srcs may
 * be peer-mapped device pointers (xGMI). dst may alias srcs[self]. */
ucs_status_t ucg_builtin_dev_reduce_multi(ucg_builtin_dev_ctx_t *ctx,
                                          ucg_dev_op_t op, ucg_dev_dtype_t dt,
                                          void *dst, const void *const *srcs,
                                          unsigned nsrc, unsigned self,
                                          size_t count);

/* One-shot tree fan-in in the association of the reference's tree plan at
 * its root (builtin/plan/builtin_tree.c:262-380 on one host: the root is the
 * only parent; init_reduce seeds the root's accumulator with its own data,
 * builtin/ops/builtin_control.c:43-47, and each child's message is reduced
 * into it as it arrives, builtin/ops/builtin_comp_step.inl:213-221):
 *   acc = srcs[0];  acc = srcs[m] (op) acc  for m = 1 .. nsrc-1
 * srcs[0] is the root's contribution and srcs[1..] the children in arrival
 * order. Any nsrc <= 16: the plan for groups that are not a power of two,
 * and for MPI_Reduce. srcs may be peer-mapped; dst may alias any source. */
ucs_status_t ucg_builtin_dev_reduce_tree(ucg_builtin_dev_ctx_t *ctx, ucg_dev_op_t op,
                                         ucg_dev_dtype_t dt, void *dst,
                                         const void *const *srcs, unsigned nsrc,
                                         size_t count);

/* ---- host-resident combine (the reduce_cb_f contract, staged) ------------*/
/* Whole-buffer: dst_host[i] = src_host[i] (op) dst_host[i]. Host chunks are
 * copied H2D into the device ring, combined and copied back D2H on two
 * streams, overlapped. An operand that is device memory is used in place (a
 * device dst is combined in place, nothing is copied back). Returns when dst
 * holds the result. */
ucs_status_t ucg_builtin_dev_combine_host(ucg_builtin_dev_ctx_t *ctx,
                                          ucg_dev_op_t op, ucg_dev_dtype_t dt,
                                          void *dst_host, const void *src_host,
                                          size_t count);

/* Per-step staging: the step's host accumulator (step->recv_buffer) is
 * mirrored on the device between stage_begin and stage_end; each fragment
 * combine copies the borrowed src into the pinned ring before returning and
 * consecutive fragments are aggregated into one launch per ring slot. */
/* host_dst may also be device memory: the step then accumulates into it in
 * place (no mirror copy either way). Fragments are always host memory (AM
 * payloads). */
ucs_status_t ucg_builtin_dev_stage_begin(ucg_builtin_dev_ctx_t *ctx,
                                         void *host_dst, size_t bytes);
ucs_status_t ucg_builtin_dev_combine(ucg_builtin_dev_ctx_t *ctx,
                                     ucg_dev_op_t op, ucg_dev_dtype_t dt,
                                     size_t dst_offset, const void *host_src,
                                     size_t count);
ucs_status_t ucg_builtin_dev_stage_end(ucg_builtin_dev_ctx_t *ctx);

/* ---- peer mapping (xGMI) for the one-shot multi-operand combine ----------*/
/* The remote key of a device buffer (the uct_md_mkey_pack of the reference's
 * zero-copy steps, builtin/ops/builtin_control.c:712-719): opaque, fixed size.
 * A key names the physical allocation, never an address:
 *  - memory of ucg_builtin_dev_malloc_shareable is mapped by a peer from the
 *    allocation's file descriptor (HIP virtual memory, POSIX fd handle),
 *    which the exporter's key server passes over a Unix socket;
 *  - any other device memory (ucg_builtin_dev_malloc, a caller's hipMalloc of
 *    an allocation of its own: not a small block the runtime carved out of a
 *    shared one) goes by hipIpcGetMemHandle, handed out only while the
 *    runtime's buffer id of the allocation at that address is the exported
 *    one.
 * Freeing an exported allocation retires its keys: a later import of one is
 * refused with UCS_ERR_NO_RESOURCE ("stale key"). A peer that mapped a
 * shareable allocation keeps its physical memory until it releases the
 * mapping, so freeing under a live importer costs no fault and hands nobody
 * else's data out. Exporting the same allocation again gives the same key.
 * The exporting process must stay alive while peers import its keys. */
#define UCG_BUILTIN_DEV_IPC_HANDLE_BYTES 96
ucs_status_t ucg_builtin_dev_ipc_export(ucg_builtin_dev_ctx_t *ctx,
                                        const void *dev_ptr, void *handle);
/* Map a peer's exported buffer into this process (once per key: a second
 * import of the same key returns the same mapping, reference counted). */
ucs_status_t ucg_builtin_dev_ipc_import(ucg_builtin_dev_ctx_t *ctx,
                                        const void *handle, void **dev_ptr);
/* Drop one import; the last one waits for the work queued on this shim's
 * contexts' streams of the device and unmaps. */
ucs_status_t ucg_builtin_dev_ipc_release(ucg_builtin_dev_ctx_t *ctx,
                                         void *dev_ptr);

/* ---- memory helpers --------------------------------------------------------*/
/* hipMalloc of whole 2 MiB granules */
void        *ucg_builtin_dev_malloc(ucg_builtin_dev_ctx_t *ctx, size_t bytes);
/* Device memory a peer maps by its physical allocation (HIP virtual memory,
 * POSIX fd handle, 2 MiB granules at a 2 MiB aligned reservation): the
 * engine's registered buffers. */
void        *ucg_builtin_dev_malloc_shareable(ucg_builtin_dev_ctx_t *ctx, size_t bytes);
/* 1 when ptr lies in a live allocation of ucg_builtin_dev_malloc_shareable */
int          ucg_builtin_dev_is_shareable(const void *ptr);
/* Frees either kind and retires the allocation's keys; a pointer of neither
 * is hipFree'd. It first waits for the work queued so far on the streams of
 * this shim's contexts on the allocation's device - not for the whole device
 * (round 6): work the caller queued on a stream of its own that uses the
 * buffer must be complete before the free, as with any stream-ordered
 * allocator. A freed
 * ucg_builtin_dev_malloc allocation is kept for the next allocation of its
 * size - one that was ever exported always (and also handed out whole for
 * a request of at least half its size), others up to
 * UCX_BUILTIN_DEV_CACHE_BYTES - so an exported address never comes back from
 * the runtime with other memory behind it. */
void         ucg_builtin_dev_free(ucg_builtin_dev_ctx_t *ctx, void *ptr);
/* For an allocation of this shim that a peer may still be reading (an op
 * that ended before every peer was done: a timeout, an error, a destroy
 * while running): retires its keys and keeps the memory allocated, never
 * handed out again, for the life of the process (ucg_builtin_dev_mem_stats
 * [6] counts it, and [7] with the other kept memory).
 *
 * Kept memory is bounded (round 6): an ucg_builtin_dev_malloc allocation is
 * kept for the life of the process from its first export on (its address
 * must never come back from the runtime with other memory behind it), and
 * ucg_builtin_dev_ipc_export fails with UCS_ERR_EXCEEDS_LIMIT when exporting
 * one more would take the kept bytes past UCX_BUILTIN_DEV_KEEP_MAX (default
 * half of the device's memory; a warning is printed once past half of it). */
void         ucg_builtin_dev_park(ucg_builtin_dev_ctx_t *ctx, void *ptr);
/* torch.cuda.memory.CUDAPluggableAllocator entry points over
 * ucg_builtin_dev_malloc_shareable / ucg_builtin_dev_free, so that every
 * tensor of a process can be exported by its physical allocation. */
void        *ucg_builtin_dev_torch_alloc(size_t bytes, int device, void *stream);
void         ucg_builtin_dev_torch_free(void *ptr, size_t bytes, int device, void *stream);
void        *ucg_builtin_dev_host_alloc(size_t bytes);      /* pinned */
void         ucg_builtin_dev_host_free(void *ptr);
/* Page-lock a caller's host buffer for DMA (hipHostRegister): the memory
 * registration of the reference's zero-copy optimisation (uct_md_mem_reg after
 * MEM_REG_OPT_CNT uses of an op, builtin_control.c:276-286, 345-373). A
 * staged step's H2D / D2H of a registered recv buffer then moves by DMA with
 * no staging copy in the runtime. The buffer must stay allocated until
 * unregistered. */
ucs_status_t ucg_builtin_dev_host_register(ucg_builtin_dev_ctx_t *ctx, void *ptr,
                                           size_t bytes);
ucs_status_t ucg_builtin_dev_host_unregister(ucg_builtin_dev_ctx_t *ctx, void *ptr);
ucs_status_t ucg_builtin_dev_memcpy(ucg_builtin_dev_ctx_t *ctx, void *dst,
                                    const void *src, size_t bytes); /* sync */
/* Occupancy cap of the multi-operand kernels (at most 12 waves per CU, by
 * their register allocation), process-wide: -1 = UCX_BUILTIN_DEV_MULTI_CAP
 * (default on), 0 = off, 1 = on. Only fp32 and fp64 SUM are built both ways;
 * every other pair always runs capped. For A/B runs inside one process
 * (bench.py's one-shot reduce-scatter over xGMI). */
void         ucg_builtin_dev_set_multi_cap(int capped);

/* Fault injection, for tests: the `after`-th call from now to a device
 * combine entry point of this process (ucg_builtin_dev_reduce, _reduce_multi,
 * _reduce_tree, _combine, _combine_host, _profile_reduce) fails with
 * UCS_ERR_IO_ERROR ("injected device error") and launches nothing; 0 disarms.
 * Returns how many injected failures have fired in this process so far. It
 * shows that a device failure on any thread - the resend timer's included -
 * reaches the operation's completion status (SURVEY.md 8b,
 * builtin_comp_step.inl:332-333). */
unsigned     ucg_builtin_dev_inject_failure(unsigned after);

/* Set the cap on kept memory (0 = back to UCX_BUILTIN_DEV_KEEP_MAX / the
 * default); for tests. */
void         ucg_builtin_dev_set_keep_max(uint64_t bytes);

/* Process-wide memory accounting of the shim (round 5, extended in round 6):
 *   [0] bytes of GPU virtual address ranges retired: a shareable allocation
 *       or an import, once unmapped, leaves its reservation behind so that no
 *       address is ever mapped to other physical memory;
 *   [1] how many such ranges;
 *   [2] the cap on [0]: past it a new shareable allocation or import fails
 *       with UCS_ERR_EXCEEDS_LIMIT (UCX_BUILTIN_DEV_VA_RETIRED_MAX, default
 *       64 TiB, or ucg_builtin_dev_set_va_retired_max);
 *   [3] bytes held by the reuse cache of freed ucg_builtin_dev_malloc
 *       allocations (its never-exported part bounded by
 *       UCX_BUILTIN_DEV_CACHE_BYTES);
 *   [4] bytes of live shareable allocations of this process;
 *   [5] bytes of live shareable imports (peers' allocations mapped here);
 *   [6] bytes parked (ucg_builtin_dev_park);
 *   [7] bytes kept for the life of the process: ever-exported
 *       ucg_builtin_dev_malloc allocations, live or cached, and parked ones;
 *   [8] the cap on [7] (UCX_BUILTIN_DEV_KEEP_MAX);
 *   [9] of [3], the ever-exported bytes;
 *   [10] slack: bytes of live allocations beyond their request (a cached
 *       ever-exported allocation handed out for a request of at least half
 *       its size). */
#define UCG_BUILTIN_DEV_NMEMSTATS 11
void         ucg_builtin_dev_mem_stats(uint64_t out[UCG_BUILTIN_DEV_NMEMSTATS]);
/* Set the cap on retired address ranges for this process (0 = back to
 * UCX_BUILTIN_DEV_VA_RETIRED_MAX / the default); for tests. */
void         ucg_builtin_dev_set_va_retired_max(uint64_t bytes);

/* Diagnostics: what the runtime and this shim know about a device address
 * (range, attributes, live or imported allocation) and the process's recent
 * memory events near it (malloc, free, export, IPC import and release),
 * as text into out[max]; returns the full length. For test harnesses that
 * find a buffer corrupted. */
size_t       ucg_builtin_dev_debug_ptr(ucg_builtin_dev_ctx_t *ctx, const void *ptr,
                                       char *out, size_t max);

/* Fill `count` elements with the counter-based synthetic generator
 * (splitmix64; identical to ucg_oracle_fill() in oracle/combine_ref.c). */
ucs_status_t ucg_builtin_dev_fill(ucg_builtin_dev_ctx_t *ctx, ucg_dev_dtype_t dt,
                                  ucg_dev_dist_t dist, uint64_t seed,
                                  void *dst, size_t count);

/* ---- profiling hooks (the UCS_PROFILE_CALL_VOID analogue, :100-101) ------*/
/* Launch `iters` back-to-back device combines between two HIP events on the
 * context stream and return the average duration of one launch in us. */
ucs_status_t ucg_builtin_dev_profile_reduce(ucg_builtin_dev_ctx_t *ctx,
                                            ucg_dev_op_t op, ucg_dev_dtype_t dt,
                                            void *dst, const void *src,
                                            size_t count, unsigned iters,
                                            double *avg_us);

/* The same for ucg_builtin_dev_reduce_multi (the one-shot reduce-scatter's
 * kernel): `iters` back-to-back launches between two HIP events. */
ucs_status_t ucg_builtin_dev_profile_reduce_multi(ucg_builtin_dev_ctx_t *ctx,
                                                  ucg_dev_op_t op, ucg_dev_dtype_t dt,
                                                  void *dst, const void *const *srcs,
                                                  unsigned nsrc, unsigned self,
                                                  size_t count, unsigned iters,
                                                  double *avg_us);

/* Measurement reference, not part of the combine path: the same launch
 * geometry (one wave per workgroup, one non-temporal 16-B vector per lane per
 * stream) streaming `bytes` bytes per stream. kind 0: read two streams (src,
 * dst) with no stores; kind 1: copy src -> dst. Average duration of one of
 * `iters` back-to-back launches in us. It gives the box's measured ceiling
 * beside the combine. bytes must be a multiple of 16 and both
 * pointers 16-B aligned. */
ucs_status_t ucg_builtin_dev_profile_stream(ucg_builtin_dev_ctx_t *ctx, int kind,
                                            void *dst, const void *src, size_t bytes,
                                            unsigned iters, double *avg_us);
/* Counters since ctx creation: [0] kernel launches, [1] bytes combined on the
 * device (3N basis), [2] H2D bytes copied by DMA (hipMemcpyAsync), [3] D2H
 * bytes, [4] staged bytes the kernel read from pinned host memory in place
 * (zero-copy runs, no DMA), [5] completion waits on the signal word. */
#define UCG_BUILTIN_DEV_NCOUNTERS 6
void         ucg_builtin_dev_counters(ucg_builtin_dev_ctx_t *ctx,
                                      uint64_t out[UCG_BUILTIN_DEV_NCOUNTERS]);

#ifdef __cplusplus
}
#endif

#endif /* UCG_BUILTIN_DEV_H_ */
