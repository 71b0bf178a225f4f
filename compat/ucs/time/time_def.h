/* compat: ucs_time_t */
#ifndef XUCG_COMPAT_UCS_TIME_DEF_H
#define XUCG_COMPAT_UCS_TIME_DEF_H
#include <stdint.h>
typedef uint64_t ucs_time_t;
#endif
