// Build provenance of liblgcn.so: the sha256 of the sources it was compiled from (every csrc
// translation unit, lgcn_common.h and include/lgcn.h, in __graft_entry__.SOURCES order), passed
// in by __graft_entry__.build() as -DLGCN_SOURCE_SHA256. lgcn_amd._ffi.load() refuses a library
// whose sources differ from the tree it is loaded from, so a test run always exercises a binary
// built from the sources next to it. The marker string also lets build() read the hash from the
// file without loading it.
#include "lgcn.h"

#ifndef LGCN_SOURCE_SHA256
#error "LGCN_SOURCE_SHA256 must be defined by the build (see __graft_entry__.build)"
#endif

#define LGCN_STR2(x) #x
#define LGCN_STR(x) LGCN_STR2(x)

extern "C" {
__attribute__((used)) static const char kMarker[] = "LGCN_SOURCE_SHA256=" LGCN_STR(LGCN_SOURCE_SHA256);

const char* lgcn_source_sha256(void) { return kMarker + 19; }
}
