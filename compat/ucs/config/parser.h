/* compat: configuration tables of <ucs/config/parser.h>: the field and
 * global-list entry types a planning component registers, the value parsers
 * its table names, and a reader that fills a component's config struct from
 * the environment (UCX_<prefix><NAME>, else the default) - what base/'s
 * ucg_plan_config_read gets from UCX's parser. */
#ifndef XUCG_COMPAT_UCS_CONFIG_PARSER_H
#define XUCG_COMPAT_UCS_CONFIG_PARSER_H

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include <ucs/config/types.h>
#include <ucs/datastruct/list.h>
#include <ucs/type/status.h>

typedef struct ucs_config_parser {
    int          (*read)(const char *buf, void *dest, const void *arg);
    int          (*write)(char *buf, size_t max, const void *src, const void *arg);
    ucs_status_t (*clone)(const void *src, void *dest, const void *arg);
    void         (*release)(void *ptr, const void *arg);
    void         (*help)(char *buf, size_t max, const void *arg);
    const void   *arg;
} ucs_config_parser_t;

typedef struct ucs_config_field {
    const char          *name;
    const char          *dfl_value;
    const char          *doc;
    size_t               offset;
    ucs_config_parser_t  parser;
} ucs_config_field_t;

typedef struct ucs_config_global_list_entry {
    const char          *name;
    const char          *prefix;
    ucs_config_field_t  *table;
    size_t               size;
    ucs_list_link_t      list;
} ucs_config_global_list_entry_t;

/* every registered table (UCS_CONFIG_REGISTER_TABLE_ENTRY); defined by the
 * library that reads the tables, weak in a component built without one */
extern ucs_list_link_t ucs_config_global_list;

#define UCS_CONFIG_REGISTER_TABLE_ENTRY(_entry) \
    UCS_STATIC_INIT { \
        ucs_list_add_tail(&ucs_config_global_list, &(_entry)->list); \
    } \
    UCS_STATIC_CLEANUP { \
        ucs_list_del(&(_entry)->list); \
    }

/* ---- value parsers ------------------------------------------------------- */
static inline UCS_F_MAYBE_UNUSED int
ucs_config_sscanf_uint(const char *buf, void *dest, const void *arg)
{
    char *end;
    unsigned long v = strtoul(buf, &end, 0);
    (void)arg;
    if (end == buf) {
        return 0;
    }
    *(unsigned*)dest = (unsigned)v;
    return 1;
}

/* a byte count with an optional k/m/g suffix, or "inf" */
static inline UCS_F_MAYBE_UNUSED int
ucs_config_sscanf_memunits(const char *buf, void *dest, const void *arg)
{
    char *end;
    double v;
    (void)arg;
    if (!strcasecmp(buf, "inf") || !strcasecmp(buf, "auto")) {
        *(size_t*)dest = UCS_MEMUNITS_INF;
        return 1;
    }
    v = strtod(buf, &end);
    if (end == buf) {
        return 0;
    }
    switch (*end) {
    case 'k': case 'K': v *= 1024.0; break;
    case 'm': case 'M': v *= 1024.0 * 1024.0; break;
    case 'g': case 'G': v *= 1024.0 * 1024.0 * 1024.0; break;
    default: break;
    }
    *(size_t*)dest = (size_t)v;
    return 1;
}

/* seconds, with an optional s/ms/us/ns suffix, stored as a double */
static inline UCS_F_MAYBE_UNUSED int
ucs_config_sscanf_time(const char *buf, void *dest, const void *arg)
{
    char *end;
    double v = strtod(buf, &end);
    (void)arg;
    if (end == buf) {
        return 0;
    }
    if (!strcmp(end, "ms")) {
        v *= 1e-3;
    } else if (!strcmp(end, "us")) {
        v *= 1e-6;
    } else if (!strcmp(end, "ns")) {
        v *= 1e-9;
    } else if (*end && strcmp(end, "s")) {
        return 0;
    }
    *(double*)dest = v;
    return 1;
}

static inline UCS_F_MAYBE_UNUSED int
ucs_config_sscanf_bool(const char *buf, void *dest, const void *arg)
{
    (void)arg;
    *(int*)dest = !strcasecmp(buf, "y") || !strcasecmp(buf, "yes") ||
                  !strcasecmp(buf, "on") || !strcmp(buf, "1");
    return 1;
}

#define UCS_CONFIG_TYPE_UINT     {ucs_config_sscanf_uint, NULL, NULL, NULL, NULL, NULL}
#define UCS_CONFIG_TYPE_MEMUNITS {ucs_config_sscanf_memunits, NULL, NULL, NULL, NULL, NULL}
#define UCS_CONFIG_TYPE_TIME     {ucs_config_sscanf_time, NULL, NULL, NULL, NULL, NULL}
#define UCS_CONFIG_TYPE_BOOL     {ucs_config_sscanf_bool, NULL, NULL, NULL, NULL, NULL}
/* a nested table: its fields are read with the outer name as a prefix */
#define UCS_CONFIG_TYPE_TABLE(_t) {NULL, NULL, NULL, NULL, NULL, _t}

/* Fill `dest` from `table`: UCX_<prefix><name> from the environment, else
 * the default. Nested tables extend the prefix. UCS_ERR_INVALID_PARAM names
 * no field: a value that does not parse. */
static inline UCS_F_MAYBE_UNUSED ucs_status_t
ucs_config_parser_fill_opts(void *dest, const ucs_config_field_t *table,
                            const char *prefix)
{
    char var[256];
    const ucs_config_field_t *f;
    for (f = table; f && f->name; f++) {
        const char *val;
        if (f->parser.read == NULL) {              /* nested table */
            char sub[128];
            ucs_status_t st;
            snprintf(sub, sizeof(sub), "%s%s", prefix, f->name);
            st = ucs_config_parser_fill_opts((char*)dest + f->offset,
                                             (const ucs_config_field_t*)f->parser.arg,
                                             sub);
            if (st != UCS_OK) {
                return st;
            }
            continue;
        }
        snprintf(var, sizeof(var), "UCX_%s%s", prefix, f->name);
        val = getenv(var);
        if (!f->parser.read(val ? val : f->dfl_value, (char*)dest + f->offset,
                            f->parser.arg)) {
            return UCS_ERR_INVALID_PARAM;
        }
    }
    return UCS_OK;
}

#endif
