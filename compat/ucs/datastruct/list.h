/* compat: intrusive doubly linked list of <ucs/datastruct/list.h> */
#ifndef XUCG_COMPAT_UCS_LIST_H
#define XUCG_COMPAT_UCS_LIST_H

#include <ucs/sys/compiler_def.h>

typedef struct ucs_list_link {
    struct ucs_list_link *prev;
    struct ucs_list_link *next;
} ucs_list_link_t;

#define UCS_LIST_INITIALIZER(_h) {&(_h), &(_h)}
#define UCS_LIST_HEAD(_name)     ucs_list_link_t _name = UCS_LIST_INITIALIZER(_name)

static inline void ucs_list_head_init(ucs_list_link_t *h)
{
    h->prev = h->next = h;
}

static inline void ucs_list_insert_after(ucs_list_link_t *pos, ucs_list_link_t *e)
{
    e->prev         = pos;
    e->next         = pos->next;
    pos->next->prev = e;
    pos->next       = e;
}

static inline void ucs_list_add_tail(ucs_list_link_t *h, ucs_list_link_t *e)
{
    ucs_list_insert_after(h->prev, e);
}

static inline void ucs_list_add_head(ucs_list_link_t *h, ucs_list_link_t *e)
{
    ucs_list_insert_after(h, e);
}

static inline void ucs_list_del(ucs_list_link_t *e)
{
    e->prev->next = e->next;
    e->next->prev = e->prev;
}

static inline int ucs_list_is_empty(const ucs_list_link_t *h)
{
    return h->next == h;
}

#define ucs_list_for_each(_elem, _head, _member) \
    for (_elem = ucs_container_of((_head)->next, __typeof__(*(_elem)), _member); \
         &(_elem)->_member != (_head); \
         _elem = ucs_container_of((_elem)->_member.next, __typeof__(*(_elem)), _member))

#define ucs_list_extract_head(_head, _type, _member) \
    ({ ucs_list_link_t *_l = (_head)->next; ucs_list_del(_l); \
       ucs_container_of(_l, _type, _member); })

#endif
