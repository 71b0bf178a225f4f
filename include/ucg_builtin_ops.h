/*
 * ucg_builtin_ops.h - the builtin planner's operation engine around the
 * combine, and a minimal host transport so a multi-process allreduce runs
 * without UCX.
 *
 * Reference anchors (paths relative to the reference tree):
 *   transport      uct_ep_am_short()/uct_iface_progress() as used by
 *                  builtin/ops/builtin_data.c:37-137 and builtin/builtin.c:
 *                  318-340; the AM data is borrowed for the callback only.
 *   wire header    ucg_builtin_header_t, builtin/ops/builtin_ops.h:53-60:
 *                  {u16 group_id; u8 coll_id; u8 step_idx; u32 remote_offset}
 *   slots          UCG_BUILTIN_MAX_CONCURRENT_OPS = 16, slot = coll_id % 16,
 *                  builtin/ops/builtin_ops.h:388, builtin/builtin.c:153-155
 *   AM handler     direct combine when local_id matches, else stash,
 *                  builtin/builtin.c:133-219
 *   step execute   send every fragment to every peer, then drain stashed
 *                  messages, builtin/ops/builtin_data.c:584-668 and
 *                  builtin/ops/builtin_comp_step.inl:403-462
 *   completion     pending = ep_cnt x fragments, next step or finish,
 *                  builtin/ops/builtin_comp_step.inl:8-95,342-401
 *   plans          recursive K-ing with its intra-host fan-in / fan-out,
 *                  builtin/plan/builtin_recursive.c:20-228; tree fan-in /
 *                  fan-out over hosts and sockets (add_intra, add_inter,
 *                  tree_connect), builtin/plan/builtin_tree.c:86-561; the
 *                  choice, builtin/builtin.c:95-121
 *   aggregation    REDUCE for REDUCE_TERMINAL/RECURSIVE/WAYPOINT, WRITE for
 *                  the fan-out receive, builtin/ops/builtin_control.c:960-972
 *                  (a REDUCE_WAYPOINT reduces here)
 *   fragments      builtin/ops/builtin_control.c:434,462-465
 *   seeding        ucg_builtin_init_reduce, builtin/ops/builtin_control.c:43-47
 *
 * Every combine goes through ucg_builtin_combine_step_begin/_fragment/
 * _step_end (include/ucg_builtin_combine.h): steps large enough and of a
 * classified type run on the device, the rest call the user's reduce_cb_f.
 */
#ifndef UCG_BUILTIN_OPS_H_
#define UCG_BUILTIN_OPS_H_

#include "ucg_builtin_combine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define UCG_BUILTIN_OPS_MAX_CONCURRENT 16   /* builtin_ops.h:388 */
#define UCG_BUILTIN_OPS_MAX_MEMBERS    64

/* ---- f2: shared-memory active-message transport ------------------------ */
typedef struct ucg_builtin_shm_iface ucg_builtin_shm_iface_t;

/* Called for every delivered message: data = 8-B header + payload,
 * `length` includes the header. The data is valid during the call only. */
typedef ucs_status_t (*ucg_builtin_am_cb_f)(void *arg, void *data, size_t length);

/* Collective over the `members` processes of one host: every member opens
 * the same `name` (a POSIX shm object, unlinked by member 0 on close).
 * max_short is the largest AM including the 8-B header (UCT cap.am.max_short;
 * the reference's BUILTIN_SHORT_MAX_TX_SIZE default is 256). */
ucs_status_t ucg_builtin_shm_iface_open(const char *name, unsigned members,
                                        unsigned my_index, size_t max_short,
                                        unsigned ring_cells,
                                        ucg_builtin_shm_iface_t **iface_p);
/* UCS_OK, or - a member's process gone, or the last barrier timed out - the
 * failure; the object is unmapped either way (never aborts the process) */
ucs_status_t ucg_builtin_shm_iface_close(ucg_builtin_shm_iface_t *iface);
size_t       ucg_builtin_shm_iface_max_short(ucg_builtin_shm_iface_t *iface);
/* The job token this process stamps into the objects it creates (the first
 * of UCX_BUILTIN_JOB_TOKEN, PMIX_NAMESPACE, OMPI_MCA_ess_base_jobid,
 * SLURM_JOB_ID:SLURM_STEP_ID, TORCHELASTIC_RUN_ID unless "none",
 * MASTER_ADDR:MASTER_PORT; 0 = none): a member refuses a live object of
 * another token. */
uint64_t     ucg_builtin_shm_job_token(void);
/* uct_ep_am_short: UCS_ERR_NO_RESOURCE when the peer's ring is full */
ucs_status_t ucg_builtin_shm_am_short(ucg_builtin_shm_iface_t *iface,
                                      unsigned peer, uint64_t header,
                                      const void *payload, size_t length);
/* uct_iface_progress: deliver pending messages; returns how many */
unsigned     ucg_builtin_shm_progress(ucg_builtin_shm_iface_t *iface,
                                      ucg_builtin_am_cb_f cb, void *arg);
/* Incast: the bcopy-into-the-root's-buffer send of the UCX collectives
 * extension that the reference's SM-root packers target (builtin/ops/
 * builtin_pack.c:50-72, 100-148; selected for SEND_TO_SM_ROOT with an
 * AGGREGATE modifier, builtin_control.c:535-602). All `expected` children
 * of `root` send the same header; the first to arrive packs with
 * reducing == 0 (copy), the rest with reducing == 1 (combine into dest) -
 * or, when `concurrent`, every child packs with reducing == 1 into a zeroed
 * cell outside the cell lock (atomic packers). The root's progress delivers
 * the cell as ONE message once all children packed. UCS_ERR_NO_RESOURCE
 * when the cell is busy with another message (retry later). */
typedef void (*ucg_builtin_pack_cb_f)(void *arg, void *dest, int reducing);
ucs_status_t ucg_builtin_shm_am_incast(ucg_builtin_shm_iface_t *iface,
                                       unsigned root, uint64_t header,
                                       unsigned expected, size_t length,
                                       ucg_builtin_pack_cb_f pack, void *arg,
                                       int concurrent);
/* The batched incast (UCX_BUILTIN_SM_INCAST=batched when the iface is
 * opened): the `expected` children of `root` each copy their message into a
 * slot of one cell of the root, and the root's progress delivers the cell as
 * ONE message of `expected` records - the reference's BATCHED_DATA receive
 * (builtin_comp_step.inl:242-273), where the root reduces every chunk itself:
 * [payload 0][header 1][payload 1]...[header n-1][payload n-1] after the
 * first header, records in arrival order. */
ucs_status_t ucg_builtin_shm_am_incast_batched(ucg_builtin_shm_iface_t *iface,
                                               unsigned root, uint64_t header,
                                               unsigned expected, const void *payload,
                                               size_t length);
/* Blocking barrier of all members (set-up / tear-down only): UCS_OK,
 * UCS_ERR_CONNECTION_RESET when a member's process is gone, UCS_ERR_TIMED_OUT
 * after UCX_BUILTIN_WAIT_TIMEOUT seconds; after a failure every later
 * barrier returns it at once. */
ucs_status_t ucg_builtin_shm_barrier(ucg_builtin_shm_iface_t *iface);

/* ---- f1: group and collective engine ------------------------------------ */
typedef struct ucg_builtin_lgroup ucg_builtin_lgroup_t;
typedef struct ucg_builtin_lcoll  ucg_builtin_lcoll_t;

/* Member distances, the values of enum ucg_group_member_distance
 * (api/ucg.h:253-264). */
#define UCG_BUILTIN_DISTANCE_SELF   0
#define UCG_BUILTIN_DISTANCE_CACHE  1
#define UCG_BUILTIN_DISTANCE_SOCKET 7
#define UCG_BUILTIN_DISTANCE_HOST   15
#define UCG_BUILTIN_DISTANCE_NET    253

/* The group's placement and the planner's tree/recursive knobs
 * (ucg_group_params_t.distance, api/ucg.h:304-324; the BUILTIN_TREE_ and
 * BUILTIN_RECURSIVE_ config tables, builtin/builtin.c:33-39,
 * builtin/plan/builtin_tree.c:18-29, builtin_recursive.c:13-18).
 *   distance    member_count entries as seen by this member (distance[my] =
 *               SELF), NULL = every other member at HOST (one host). Members
 *               of a host carry consecutive indices and every host the same
 *               number of them (the reference's "by node" allocation,
 *               builtin_tree.c:397-405); other layouts are UCS_ERR_UNSUPPORTED.
 *               The transport stays the shared-memory one: a NET distance
 *               changes the plan, not the wire, so multi-host plans run on
 *               one machine.
 *   tree_radix  UCX_BUILTIN_TREE_RADIX (0 = environment, else 8): fan-out of
 *               the inter-host tree
 *   sock_thresh UCX_BUILTIN_TREE_SOCKET_LEVEL_PPN_THRESH (0 = environment,
 *               else 16): from this many members per host on, SOCKET
 *               distances make a second intra-host tree level
 *   recursive_factor UCX_BUILTIN_RECURSIVE_FACTOR (0 = environment, else 2):
 *               the K of recursive K-ing */
typedef struct ucg_builtin_lgroup_params {
    const uint8_t *distance;
    unsigned       tree_radix;
    unsigned       sock_thresh;
    unsigned       recursive_factor;
    int            mem_reg_opt_cnt;   /* BUILTIN_MEM_REG_OPT_CNT (builtin.c:49-50):
                                         0 = UCX_BUILTIN_MEM_REG_OPT_CNT (10),
                                         > 0 = that many starts, < 0 = never */
} ucg_builtin_lgroup_params_t;

/* group_id must be non-zero (builtin_control.c:645 asserts it; the plan
 * component maps a caller's group id 0 to an internal one); `combine` is the
 * per-group combine state and stays owned by the caller. */
ucs_status_t ucg_builtin_lgroup_create(ucg_builtin_shm_iface_t *iface,
                                       uint16_t group_id, unsigned member_count,
                                       unsigned my_index,
                                       ucg_builtin_combine_t *combine,
                                       ucg_builtin_lgroup_t **group_p);
/* The same with a placement and planner knobs (NULL params = the call
 * above). */
ucs_status_t ucg_builtin_lgroup_create_ex(ucg_builtin_shm_iface_t *iface,
                                          uint16_t group_id, unsigned member_count,
                                          unsigned my_index,
                                          ucg_builtin_combine_t *combine,
                                          const ucg_builtin_lgroup_params_t *params,
                                          ucg_builtin_lgroup_t **group_p);
void         ucg_builtin_lgroup_destroy(ucg_builtin_lgroup_t *group);
/* Progress the transport and any pending resends of this group's ops. */
unsigned     ucg_builtin_lgroup_progress(ucg_builtin_lgroup_t *group);
/* The resend timer of the group's async context (RESEND_TIMER_TICK,
 * builtin/builtin.c:55-56, 284-294, 408-413): every interval_s a thread of its
 * own retries the sends of every op that stopped at UCS_ERR_NO_RESOURCE, as
 * progress does; a step whose sends then complete drains what is stashed for
 * it, so the combine may run on that thread ("Thread
 * boundary"). Every entry point of the group takes the group's lock, as the
 * reference's UCS_ASYNC_BLOCK. Stopped by lgroup_destroy. */
ucs_status_t ucg_builtin_lgroup_set_async_timer(ucg_builtin_lgroup_t *group,
                                                double interval_s);
/* [0] resends made by the timer thread, [1] fragments it combined */
void         ucg_builtin_lgroup_async_stats(ucg_builtin_lgroup_t *group, uint64_t out[2]);

/* MPI_Allreduce (modifiers AGGREGATE|BROADCAST, api/ucg_mpi.h:53-54), the
 * plan ucg_builtin_choose_topology picks (builtin/builtin.c:112-121):
 *  - member_count a power of two: the recursive plan (builtin_recursive.c:
 *    20-228): recursive K-ing over the hosts' masters (peers my^... for K=2,
 *    K-1 peers per step otherwise), wrapped in an intra-host fan-in/fan-out
 *    when a host has several members; one host whose size is not a power of
 *    K falls back to the intra-host tree; several hosts whose number is not
 *    a power of K are UCS_ERR_UNSUPPORTED (:77-88).
 *  - otherwise the tree (builtin_tree.c:441-523): intra-host fan-in to each
 *    host's master (two levels from sock_thresh members per host), the
 *    inter-host tree of `tree_radix` over the masters, and the fan-out back.
 * UCX_BUILTIN_ALLREDUCE_PLAN=tree|recursive overrides the choice (a knob of
 * this build). sbuf == rbuf means in place. The op is reusable (persistent).
 *
 * Device buffers (GPU memory, with a device attached to the combine): the same
 * plan runs as remote-key steps - the reference's rkey exchange and zero-copy
 * reads (builtin_control.c:1014-1076, builtin_data.c:326-340). Each member
 * keeps its data in two registered device buffers of the group's pool, sends
 * their IPC keys once per op to the members that read from it, and a step
 * becomes READY (to the readers) and one kernel over the senders' buffers
 * followed by DONE (to the senders). Every member must pass device buffers
 * (one host and one device buffer is UCS_ERR_UNSUPPORTED), and the transport
 * must carry 112-byte messages. The (op, dtype) must classify for the device. */
ucs_status_t ucg_builtin_lcoll_allreduce(ucg_builtin_lgroup_t *group,
                                         const void *sbuf, void *rbuf,
                                         int count, void *dtype, void *op,
                                         ucg_builtin_lcoll_t **coll_p);
/* MPI_Reduce (AGGREGATE|SINGLE_DESTINATION, api/ucg_mpi.h:41-42, 156): the
 * tree's fan-in to `root`, whose rbuf receives the result; rbuf is not
 * touched (may be NULL) on the other members - a member that combines on
 * the way (a host master, a waypoint) uses a buffer of the op's own. A root
 * other than 0 takes the tree built for root 0 with its host moved to the
 * front and the root to the front of its host. */
ucs_status_t ucg_builtin_lcoll_reduce(ucg_builtin_lgroup_t *group,
                                      const void *sbuf, void *rbuf,
                                      int count, void *dtype, void *op,
                                      unsigned root, ucg_builtin_lcoll_t **coll_p);
/* Up to UCG_BUILTIN_OPS_MAX_CONCURRENT ops of a group may be in flight. One
 * REDUCE step at a time holds the combine's step staging (device mirror);
 * a step that finds it busy combines each fragment on its own through
 * ucg_builtin_combine_reduce (the reference's per-fragment call). */
/* Registered memory of the group (the memory registration the reference's
 * zero-copy steps rely on, ucg_builtin_step_zcopy_prep, builtin_control.c:
 * 276-286): device memory (on_device, needs a device on the combine) or a
 * POSIX shared-memory segment. Used as an op's send buffer (not in place), a
 * remote-key step exposes it where it is instead of copying it into the op's
 * own buffer first. Stays registered until the group is destroyed; mem_free
 * returns it to the group's pool. NULL on failure. */
void        *ucg_builtin_lgroup_mem_alloc(ucg_builtin_lgroup_t *group, size_t bytes,
                                          int on_device);
void         ucg_builtin_lgroup_mem_free(ucg_builtin_lgroup_t *group, void *ptr);
/* ucg_collective_start: UCS_OK if complete, UCS_INPROGRESS, or an error */
ucs_status_t ucg_builtin_lcoll_start(ucg_builtin_lcoll_t *coll);
/* The same under the collective id base/ hands out (ucg_collective_trigger,
 * base/ucg_group.c:485-500; ucg_builtin_op_trigger, builtin_control.c:
 * 1309-1352): every member must start the op under the same id.
 * UCS_ERR_BUSY when the id's slot (coll_id % 16) still runs an op. */
ucs_status_t ucg_builtin_lcoll_start_as(ucg_builtin_lcoll_t *coll, uint8_t coll_id);
/* 1 when the last start completed; its status in *status */
int          ucg_builtin_lcoll_test(ucg_builtin_lcoll_t *coll,
                                    ucs_status_t *status);
/* Progress until complete (or error); returns the final status. */
ucs_status_t ucg_builtin_lcoll_wait(ucg_builtin_lcoll_t *coll);
void         ucg_builtin_lcoll_destroy(ucg_builtin_lcoll_t *coll);
/* ucg_params_t.completion (api/ucg.h:162-171), called where the reference's
 * ucg_builtin_comp_last_step_cb calls it (builtin_comp_step.inl:8-38): when a
 * start completes - from lcoll_start itself, or from progress - cb(req,
 * status) runs; with cb NULL, a 1 byte is written at req + flag_offset and the
 * status (ucs_status_t) at req + status_offset. Also called with
 * UCS_ERR_CANCELED when an op still running is destroyed. The callback runs
 * inside the engine: it may record the completion, not restart or destroy
 * the op. */
typedef void (*ucg_builtin_coll_comp_cb_f)(void *req, ucs_status_t status);
ucs_status_t ucg_builtin_lcoll_set_completion(ucg_builtin_lcoll_t *coll,
                                              ucg_builtin_coll_comp_cb_f cb, void *req,
                                              size_t flag_offset, size_t status_offset);
/* The plan as the builtin planner's print (builtin/builtin.c:750-901):
 * steps, peers, fragment length and count. Returns bytes written. */
size_t       ucg_builtin_lcoll_describe(ucg_builtin_lcoll_t *coll, char *buf,
                                        size_t max);
/* [0] messages sent, [1] messages received directly, [2] stashed,
 * [3] resends after UCS_ERR_NO_RESOURCE */
void         ucg_builtin_lgroup_stats(ucg_builtin_lgroup_t *group,
                                      uint64_t out[4]);

#ifdef __cplusplus
}
#endif

#endif
