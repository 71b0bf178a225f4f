/* compat: the recursive spinlock ucg_plan_t embeds */
#ifndef XUCG_COMPAT_UCS_SPINLOCK_H
#define XUCG_COMPAT_UCS_SPINLOCK_H

#include <pthread.h>
#include <ucs/type/status.h>

typedef struct ucs_spinlock {
    pthread_spinlock_t lock;
} ucs_spinlock_t;

typedef struct ucs_recursive_spinlock {
    ucs_spinlock_t super;
    int            count;
    pthread_t      owner;
} ucs_recursive_spinlock_t;

static inline ucs_status_t
ucs_recursive_spinlock_init(ucs_recursive_spinlock_t *l, int flags)
{
    (void)flags;
    l->count = 0;
    l->owner = (pthread_t)0;
    return pthread_spin_init(&l->super.lock, PTHREAD_PROCESS_PRIVATE) ?
           UCS_ERR_IO_ERROR : UCS_OK;
}

static inline void ucs_recursive_spinlock_destroy(ucs_recursive_spinlock_t *l)
{
    pthread_spin_destroy(&l->super.lock);
}

#endif
