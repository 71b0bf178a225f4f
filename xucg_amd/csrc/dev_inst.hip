/*
 * dev_inst.hip - the kernels and launchers of ONE dtype (UCG_INST_DT),
 * compiled once per dtype by the Makefile so the 96 (dtype, op) pairs build
 * in parallel. See dev_launch.h.
 */
#include "dev_launch.h"

#ifndef UCG_INST_DT
#error "compile with -DUCG_INST_DT=<ucg_dev_dtype_t value>"
#endif

namespace ucgdev {
template <>
RowSet rows<UCG_INST_DT>()
{
    return make_rows<UCG_INST_DT>();
}
}  // namespace ucgdev
