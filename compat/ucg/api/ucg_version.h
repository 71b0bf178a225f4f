/* compat: stands in for the file autotools generates from the reference's
 * api/ucg_version.h.in (version 1.0 of the UCG API) */
#ifndef XUCG_COMPAT_UCG_VERSION_H
#define XUCG_COMPAT_UCG_VERSION_H
#define UCG_VERSION_MAJOR_SHIFT 24
#define UCG_VERSION_MINOR_SHIFT 16
#define UCG_VERSION(_major, _minor) \
    (((_major) << UCG_VERSION_MAJOR_SHIFT) | ((_minor) << UCG_VERSION_MINOR_SHIFT))
#define UCG_API_MAJOR   1
#define UCG_API_MINOR   0
#define UCG_API_VERSION UCG_VERSION(1, 0)
#endif
