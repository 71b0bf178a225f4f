/* compat: singly linked queue element of <ucs/datastruct/queue_types.h> */
#ifndef XUCG_COMPAT_UCS_QUEUE_TYPES_H
#define XUCG_COMPAT_UCS_QUEUE_TYPES_H

typedef struct ucs_queue_elem {
    struct ucs_queue_elem *next;
} ucs_queue_elem_t;

typedef struct ucs_queue_head {
    ucs_queue_elem_t  *head;
    ucs_queue_elem_t **ptail;
} ucs_queue_head_t;

#endif
