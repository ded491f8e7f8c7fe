// Host-only stand-ins for the two runtime.hip entry points the host C++ files call, so that
// binfile.cpp and host_post.cpp build without HIP into the sanitizer library of `make asan`
// (libwavernn_host_asan.so: ASan + UBSan over the .bin reader and the post-processing loops).
// Not part of the product library.
#include <string>

#include "wavernn_mi355x.h"

namespace {
thread_local std::string g_err;
}

extern "C" int wrnn_internal_fail(int code, const char* msg) {
    g_err = msg ? msg : "";
    return code;
}

extern "C" const char* wrnn_last_error(void) { return g_err.c_str(); }

extern "C" const char* wrnn_version(void) { return "wavernn-mi355x host-only sanitizer build"; }
