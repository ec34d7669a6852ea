// Build provenance of libfa_host.so: FA_BUILD_ID is the hash of the sources and flags
// this library was compiled from (ops/build.py source_id), passed with -D by the build.
// The marker string also lets the build read the id from the file without loading it.
#include "fa_common.h"

#ifndef FA_BUILD_ID
#define FA_BUILD_ID "unknown"
#endif

static const char kBuildMarker[] __attribute__((used)) = "FA_BUILD_ID:" FA_BUILD_ID;

FA_API const char* fa_build_id() { return kBuildMarker + 12; }
