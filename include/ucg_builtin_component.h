/*
 * ucg_builtin_component.h - builtin-private additions to the plan component
 * (not part of api/): the drop-in itself is the global `ucg_builtin_component`
 * that libucg_builtin.so exports (xucg_amd/csrc/builtin_component.c), of type
 * ucg_plan_component_t (api/ucg_plan_component.h:141-188; this build's
 * declaration: include/ucg_api_abi.h).
 *
 * api/ cannot tell MAX from MIN or PROD, nor fp16 from bf16 (it offers
 * is_sum_f and the integer / floating-point / size queries only,
 * api/ucg.h:129-160). An MPI integration that wants those on the device
 * registers its classifier here once, before groups are created; every group's
 * combine then uses it. Without it, SUM and the types the
 * callbacks identify run on the device, everything else on reduce_cb_f.
 */
#ifndef UCG_BUILTIN_COMPONENT_H_
#define UCG_BUILTIN_COMPONENT_H_

#include "ucg_builtin_combine.h"

#ifdef __cplusplus
extern "C" {
#endif

void ucg_builtin_component_set_classifier(ucg_builtin_op_classifier_f op_cls,
                                          ucg_builtin_dt_classifier_f dt_cls);

/* The vtable's destroy returns nothing (api/ucg_plan_component.h:161-162),
 * yet a group's tear-down can fail: a member's process gone
 * (UCS_ERR_CONNECTION_RESET) or its last barrier timed out. destroy then
 * still frees everything, warns on stderr and keeps the status here: the
 * status of the last group destroy of this process (UCS_OK if none failed). */
ucs_status_t ucg_builtin_component_last_destroy_status(void);

#ifdef __cplusplus
}
#endif

#endif
