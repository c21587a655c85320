/* wrapper.h -- byte-for-byte the reference's cgo-facing declaration
 * (/root/reference/wrapper.h:1-13).  libcld_mi355x.so exports this symbol, so
 * the Go service's `#include "wrapper.h"` + `-lcld_mi355x` keeps compiling
 * unchanged. */
#ifndef __WRAPPER_H
#define __WRAPPER_H

#ifdef __cplusplus
extern "C" {
#endif

const char* detect_language(const char *text);

#ifdef __cplusplus
}
#endif
#endif
