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

// ---- measurement infrastructure: an emulated collective (bench.py --simulate-world) --------------
// One rank's share of the sharded step runs on one GPU with each RCCL collective replaced by this
// kernel on the stream the collective would be issued on: `workgroups` workgroups of `threads`
// threads that stay resident for `us` microseconds of wall time (the steady 100 MHz counter), so a
// captured step shows the modeled collective's duration, its ordering against the kernels around
// it (overlap on a side / comm stream) and the CU slots an RCCL kernel would hold (contention).
// Every wave leaves once its own clock passes the deadline: the grid always drains.
__global__ __launch_bounds__(1024) void sim_collective_kernel(long long ticks) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int hicgat_sim_collective(float us, int workgroups, int threads, hicgat_stream_t stream) {
  if (!(us >= 0.f) || us > 1e6f || workgroups < 1 || workgroups > 4096 || threads < 64 || threads > 1024 ||
      threads % 64)
    return HICGAT_EINVAL;
  static int khz = 0;   // the steady counter's rate (kHz): 100 MHz on MI300-class parts
  if (khz == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) !=
                                                hipSuccess || v <= 0)
      return HICGAT_ELAUNCH;
    khz = v;
  }
  const long long ticks = (long long)((double)us * 1e-3 * (double)khz);
  hipLaunchKernelGGL(sim_collective_kernel, dim3(workgroups), dim3(threads), 0, (hipStream_t)stream, ticks);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}

// ---- streams and stamps -------------------------------------------------------------------------
extern "C" int hicgat_stream_create(int priority, hicgat_stream_t *out) {
  if (!out) return HICGAT_EINVAL;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority) != hipSuccess) return HICGAT_ELAUNCH;
  *out = (hicgat_stream_t)s;
  return HICGAT_OK;
}

// one wave; lane 0 writes (a per-lane vector store, like every other store of the library)
__global__ __launch_bounds__(64) void wall_stamp_kernel(unsigned long long *out, int slot) {
  const unsigned long long t = wall_clock64();
  if (threadIdx.x == 0) out[slot] = t;
}

extern "C" int hicgat_wall_stamp(unsigned long long *out, int slot, hicgat_stream_t stream) {
  if (!out || slot < 0 || (reinterpret_cast<uintptr_t>(out) & 7)) return HICGAT_EINVAL;
  hipLaunchKernelGGL(wall_stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out, slot);
  HICGAT_CHECK_LAUNCH();
  return HICGAT_OK;
}
