// qoc_version.hip — qoc_source_hash(): the sha256 of the sources this library was built from (__graft_entry__.build_lib
// passes it as QOC_SOURCE_HASH; qoc_amd._lib.load refuses a library whose hash differs from the tree).  Its own
// translation unit, so that a new hash recompiles only this file.
#include "../../include/qoc.h"

#ifndef QOC_SOURCE_HASH
#define QOC_SOURCE_HASH "unknown"
#endif

extern "C" const char* qoc_source_hash(void) { return QOC_SOURCE_HASH; }
