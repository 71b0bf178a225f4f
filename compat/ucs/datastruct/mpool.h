/* compat: the memory-pool handle (the API headers only include it) */
#ifndef XUCG_COMPAT_UCS_MPOOL_H
#define XUCG_COMPAT_UCS_MPOOL_H
typedef struct ucs_mpool ucs_mpool_t;
#endif
