// Library identity and error strings of libhicgat.so.
#include "common.hpp"

extern "C" int hicgat_version(void) { return 1; }

extern "C" const char *hicgat_strerror(int code) {
  switch (code) {
    case HICGAT_OK: return "ok";
    case HICGAT_EINVAL: return "invalid argument (size, null pointer, workspace or alignment)";
    case HICGAT_ELAUNCH: return "kernel launch failed (hipGetLastError)";
    case HICGAT_EUNSUPPORTED: return "unsupported shape for this kernel";
    default: return "unknown hicgat error";
  }
}
