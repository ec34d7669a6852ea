// Build provenance of libfa_hip.so: FA_BUILD_ID is the hash of the kernel sources and
// the hipcc flags (ops/build.py source_id), passed with -D by the build; the marker
// string lets the build read the id from the file without loading the library.
#include "fa_hip.h"

#ifndef FA_BUILD_ID
#define FA_BUILD_ID "unknown"
#endif

static const char kBuildMarker[] __attribute__((used)) = "FA_BUILD_ID:" FA_BUILD_ID;

FA_API const char* fa_build_id() { return kBuildMarker + 12; }
