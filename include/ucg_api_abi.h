/*
 * ucg_api_abi.h - the part of UCG's public and plan-component API that the
 * builtin planner exchanges with base/, declared for this build.
 *
 * The drop-in boundary of this repository is the plan component: the global
 * `ucg_builtin_component` of type ucg_plan_component_t, which base/
 * (ucg_plan.c, ucg_group.c) finds in ucg_plan_components_list and drives
 * through its vtable. That type, and every type it passes - the collective
 * parameters, plans, operations, group parameters and the process-global
 * ucg_params_t the combine callbacks come from - are declared here with the
 * layout of the reference's headers:
 *
 *   ucg_def.h types              api/ucg_def.h:35-132
 *   ucg_params_t                 api/ucg.h:92-184
 *   collective modifiers         api/ucg.h:208-226
 *   ucg_collective_type_t        api/ucg.h:239-243
 *   member distances             api/ucg.h:253-265
 *   ucg_group_params_t           api/ucg.h:274-325
 *   ucg_collective_params_t      api/ucg.h:337-369
 *   plan/op/desc types           api/ucg_plan_component.h:26-139
 *   ucg_plan_component_t         api/ucg_plan_component.h:141-188
 *   UCG_PLAN_COMPONENT_DEFINE    api/ucg_plan_component.h:190-249
 *
 * Inside a UCG tree builtin_component.c includes the reference's own
 * <ucg/api/ucg_plan_component.h> instead (XUCG_REFERENCE_API);
 * tests/test_component.py compiles the unchanged reference headers over
 * compat/ and checks every offset and size below against them. The UCX types
 * come from compat/ (or UCX itself).
 */
#ifndef UCG_API_ABI_H_
#define UCG_API_ABI_H_

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include <ucs/config/parser.h>
#include <ucs/datastruct/list.h>
#include <ucs/datastruct/queue_types.h>
#include <ucs/sys/compiler_def.h>
#include <ucs/type/spinlock.h>
#include <ucs/type/status.h>
#include <ucp/api/ucp.h>
#include <uct/api/uct.h>

BEGIN_C_DECLS

/* ---- api/ucg_def.h ------------------------------------------------------ */
typedef struct ucg_context *ucg_context_h;
typedef struct ucg_config   ucg_config_t;
typedef struct ucg_group   *ucg_group_h;
typedef void               *ucg_coll_h;
typedef uint16_t            ucg_group_id_t;
typedef uint64_t            ucg_group_member_index_t;
typedef void     (*ucg_collective_callback_t)(void *request, ucs_status_t status);
typedef unsigned (*ucg_collective_progress_t)(ucg_coll_h coll);

/* ---- api/ucg.h ---------------------------------------------------------- */
enum ucg_params_field {
    UCG_PARAM_FIELD_JOB_UID       = UCS_BIT(0),
    UCG_PARAM_FIELD_ADDRESS_CB    = UCS_BIT(1),
    UCG_PARAM_FIELD_NEIGHBORS_CB  = UCS_BIT(2),
    UCG_PARAM_FIELD_DATATYPE_CB   = UCS_BIT(3),
    UCG_PARAM_FIELD_REDUCE_OP_CB  = UCS_BIT(4),
    UCG_PARAM_FIELD_COMPLETION_CB = UCS_BIT(5),
    UCG_PARAM_FIELD_MPI_IN_PLACE  = UCS_BIT(6),
    UCG_PARAM_FIELD_HANDLE_FAULT  = UCS_BIT(7)
};

enum ucg_fault_tolerance_mode {
    UCG_FAULT_IS_FATAL = 0,
    UCG_FAULT_IS_RETURNED,
    UCG_FAULT_IS_TRANSPARENT,
    UCG_FAULT_IS_HANDLED_BY_USER
};

/* the process-wide parameters; the builtin planner reads the datatype and
 * reduce_op callbacks (the combine, reduce_cb_f) and the completion */
typedef struct ucg_params {
    ucp_params_t *super;
    uint64_t      field_mask;
    uint32_t      job_uid;
    struct {
        int  (*lookup_f)(void *cb_group_context, ucg_group_member_index_t index,
                         ucp_address_t **addr, size_t *addr_len);
        void (*release_f)(ucp_address_t *addr);
    } address;
    struct {
        int (*vertex_count_f)(void *cb_group_context, unsigned *in_degree,
                              unsigned *out_degree);
        int (*vertex_query_f)(void *cb_group_context, ucg_group_member_index_t *in,
                              ucg_group_member_index_t *out);
    } neighbors;
    struct {
        int (*convert)(void *datatype, ucp_datatype_t *ucp_datatype);
        int (*is_integer_f)(void *datatype, int *is_signed);
        int (*is_floating_point_f)(void *datatype);
    } datatype;
    struct {
        int (*reduce_cb_f)(void *reduce_op, char *src, char *dst, unsigned count,
                           void *datatype);
        int (*is_sum_f)(void *reduce_op);
        int (*is_loc_expected_f)(void *reduce_op);
        int (*is_commutative_f)(void *reduce_op);
    } reduce_op;
    struct {
        void   (*coll_comp_cb_f)(void *req, ucs_status_t status);
        size_t comp_flag_offset;
        size_t comp_status_offset;
    } completion;
    void *mpi_in_place;
    struct {
        enum ucg_fault_tolerance_mode mode;
        void *context;
        int  (*handler_f)(void *context, int *error_code, ...);
        void (*err_str_f)(int error_code, char **error_description);
    } fault;
} ucg_params_t;

enum ucg_collective_modifiers {
    UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_SOURCE      = UCS_BIT(0),
    UCG_GROUP_COLLECTIVE_MODIFIER_SINGLE_DESTINATION = UCS_BIT(1),
    UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE          = UCS_BIT(2),
    UCG_GROUP_COLLECTIVE_MODIFIER_CONCATENATE        = UCS_BIT(3),
    UCG_GROUP_COLLECTIVE_MODIFIER_BROADCAST          = UCS_BIT(4),
    UCG_GROUP_COLLECTIVE_MODIFIER_VARIADIC           = UCS_BIT(5),
    UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE_PARTIAL  = UCS_BIT(6),
    UCG_GROUP_COLLECTIVE_MODIFIER_NEIGHBOR           = UCS_BIT(7),
    UCG_GROUP_COLLECTIVE_MODIFIER_AGGREGATE_STABLE   = UCS_BIT(8),
    UCG_GROUP_COLLECTIVE_MODIFIER_NONCONTIG_DATATYPE = UCS_BIT(9),
    UCG_GROUP_COLLECTIVE_MODIFIER_PERSISTENT         = UCS_BIT(10),
    UCG_GROUP_COLLECTIVE_MODIFIER_SYMMETRIC          = UCS_BIT(11),
    UCG_GROUP_COLLECTIVE_MODIFIER_BARRIER            = UCS_BIT(12),
    UCG_GROUP_COLLECTIVE_MODIFIER_MOCK_EPS           = UCS_BIT(13)
};

typedef struct ucg_collective_type {
    uint16_t                 modifiers;
    ucg_group_member_index_t root :48;
} UCS_S_PACKED ucg_collective_type_t;

enum ucg_group_member_distance {
    UCG_GROUP_MEMBER_DISTANCE_SELF   = 0,
    UCG_GROUP_MEMBER_DISTANCE_CACHE  = UCS_MASK(1),
    UCG_GROUP_MEMBER_DISTANCE_SOCKET = UCS_MASK(3),
    UCG_GROUP_MEMBER_DISTANCE_HOST   = UCS_MASK(4),
    UCG_GROUP_MEMBER_DISTANCE_NET    = UCS_MASK(8) - 2,
    UCG_GROUP_MEMBER_DISTANCE_FAULT  = UCS_MASK(8) - 1,
    UCG_GROUP_MEMBER_DISTANCE_LAST   = UCS_MASK(8)
} UCS_S_PACKED;

enum ucg_group_params_field {
    UCG_GROUP_PARAM_FIELD_ID           = UCS_BIT(0),
    UCG_GROUP_PARAM_FIELD_MEMBER_COUNT = UCS_BIT(1),
    UCG_GROUP_PARAM_FIELD_MEMBER_INDEX = UCS_BIT(2),
    UCG_GROUP_PARAM_FIELD_CB_CONTEXT   = UCS_BIT(3),
    UCG_GROUP_PARAM_FIELD_DISTANCES    = UCS_BIT(4)
};

typedef struct ucg_group_params {
    uint64_t                        field_mask;
    ucg_group_id_t                  id;
    ucg_group_member_index_t        member_count;
    ucg_group_member_index_t        member_index;
    void                           *cb_context;
    enum ucg_group_member_distance *distance;
} ucg_group_params_t;

/* 64 bytes: base/ucg_group.c:410-423 compares whole cache lines of these */
typedef struct ucg_collective {
    struct {
        union {
            ucg_collective_type_t type;     /* send only */
            void                 *op;       /* recv only: the reduce_op handle */
            const int            *displs;
        };
        void *buffer;
        union {
            int64_t    count;
            const int *counts;
        };
        union {
            void *dtype;
            void *dtypes;
        };
    } send, recv;
} UCS_S_PACKED UCS_V_ALIGNED(64) ucg_collective_params_t;

#define UCG_PARAM_TYPE(_params)   (_params)->send.type
#define UCG_PARAM_OP(_params)     (_params)->recv.op
#define UCG_PARAM_DISPLS(_params) (_params)->recv.displs

/* ---- api/ucg_plan_component.h ------------------------------------------- */
typedef uint8_t                   ucg_coll_id_t;
typedef uint8_t                   ucg_step_idx_t;
typedef uint32_t                  ucg_offset_t;
typedef void                     *ucg_plan_ctx_h;
typedef void                     *ucg_group_ctx_h;
typedef struct ucg_plan_config    ucg_plan_config_t;
typedef struct ucg_plan_component ucg_plan_component_t;

extern ucs_list_link_t ucg_plan_components_list;
extern ucg_params_t    ucg_global_params;

typedef struct ucg_plan_plogp_params {
    struct {
        double sec_per_message;
        double sec_per_byte;
    } send, recv, gap;
    double                   latency_in_sec[UCG_GROUP_MEMBER_DISTANCE_LAST];
    ucg_group_member_index_t peer_count[UCG_GROUP_MEMBER_DISTANCE_LAST];
} ucg_plan_plogp_params_t;

typedef double (*ucg_plan_estimator_f)(ucg_plan_plogp_params_t plogp,
                                       ucg_collective_params_t *coll);

enum ucg_plan_flags {
    UCG_PLAN_FLAG_PLOGP_LATENCY_ESTIMATOR = 0,
    UCG_PLAN_FLAG_FAULT_TOLERANCE_SUPPORT = 1
};

#define UCG_PLAN_COMPONENT_NAME_MAX (16)
typedef struct ucg_plan_desc {
    char                  name[UCG_PLAN_COMPONENT_NAME_MAX];
    ucg_plan_component_t *component;
    unsigned              modifiers_supported;
    unsigned              flags;
    ucg_plan_estimator_f  latency_estimator;
    unsigned              fault_tolerance_supported;
} ucg_plan_desc_t;

typedef struct ucg_plan_params {
    uint8_t *am_id;           /* active-message id dispenser */
} ucg_plan_params_t;

/* filled by base/ucg_group.c:82-100 after the component's plan() */
typedef struct ucg_plan {
    ucs_recursive_spinlock_t lock;
    ucs_list_link_t          op_head;
    ucg_plan_desc_t         *planner;
    ucg_group_id_t           group_id;
    ucg_group_member_index_t group_size;
    ucg_group_member_index_t my_index;
    ucg_group_h              group;
    char                     priv[0];
} ucg_plan_t;

typedef struct ucg_op ucg_op_t;
typedef ucs_status_t (*ucg_op_trigger_f)(ucg_op_t *op, ucg_coll_id_t coll_id,
                                         void *request);
typedef void         (*ucg_op_discard_f)(ucg_op_t *op);

struct ucg_op {
    ucg_op_trigger_f trigger_f;
    ucg_op_discard_f discard_f;
    union {
        ucs_list_link_t list;            /* base's op cache */
        struct {
            ucs_queue_elem_t queue;      /* base's barrier-pending queue */
            void            *pending_req;
        };
    };
    ucg_plan_t              *plan;
    ucg_collective_params_t  params;     /* 64-byte aligned */
    char                     priv[0];
};

struct ucg_plan_component {
    const char                     name[UCG_PLAN_COMPONENT_NAME_MAX];
    ucs_config_global_list_entry_t config;
    size_t                         global_ctx_size;
    size_t                         per_group_ctx_size;
    ucs_list_link_t                list;

    ucs_status_t (*query)(ucg_plan_desc_t *descs, unsigned *desc_cnt_p);
    ucs_status_t (*init)(ucg_plan_ctx_h ctx, ucg_plan_params_t *params,
                         ucg_plan_config_t *config);
    void         (*finalize)(ucg_plan_ctx_h ctx);
    ucs_status_t (*create)(ucg_plan_ctx_h ctx, ucg_group_ctx_h gctx, ucg_group_h group,
                           const ucg_group_params_t *group_params);
    void         (*destroy)(ucg_group_ctx_h gctx);
    ucs_status_t (*plan)(ucg_group_ctx_h gctx, const ucg_collective_type_t *coll_type,
                         ucg_plan_t **plan_p);
    ucs_status_t (*prepare)(ucg_plan_t *plan, const ucg_collective_params_t *coll_params,
                            ucg_op_t **op);
    ucg_op_trigger_f          trigger;
    ucg_collective_progress_t progress;
    ucg_op_discard_f          discard;
    void         (*print)(ucg_plan_t *plan, const ucg_collective_params_t *coll_params);
    ucs_status_t (*fault)(ucg_group_ctx_h gctx, ucg_group_member_index_t index);
};

/* the component object, self-registered into ucg_plan_components_list at load
 * time, with its configuration table registered for UCX's parser */
#define UCG_PLAN_COMPONENT_DEFINE(_planc, _name, _global_size, _group_size,        \
                                  _query, _init, _finalize, _create, _destroy,     \
                                  _plan, _prepare, _trigger, _progress, _discard,  \
                                  _print, _fault, _cfg_prefix, _cfg_table,         \
                                  _cfg_struct)                                     \
    ucg_plan_component_t _planc = {                                                \
        .name = _name,                                                             \
        .config = {.name = _name " planner", .prefix = _cfg_prefix,                \
                   .table = _cfg_table, .size = sizeof(_cfg_struct)},              \
        .global_ctx_size = _global_size, .per_group_ctx_size = _group_size,        \
        .query = _query, .init = _init, .finalize = _finalize,                     \
        .create = _create, .destroy = _destroy, .plan = _plan,                     \
        .prepare = _prepare, .trigger = _trigger, .progress = _progress,           \
        .discard = _discard, .print = _print, .fault = _fault};                   \
    UCS_STATIC_INIT {                                                              \
        ucs_list_add_tail(&ucg_plan_components_list, &(_planc).list);             \
    }                                                                              \
    UCS_CONFIG_REGISTER_TABLE_ENTRY(&(_planc).config)

END_C_DECLS

#endif
