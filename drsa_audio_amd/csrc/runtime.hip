// Host-side runtime helpers shared by every launch site of libdrsa_amd (gfx950).
//
// * per-thread error message behind drsa_amd_last_error()
// * ensure_smem(): hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel,
//   size) — per device, because the attribute lives in the device's context, and under a mutex,
//   because the C ABI may be called from several host threads (the reference drives rules from
//   the autograd thread).
// * cu_count(): multiprocessor count of the CURRENT device (cached per device).
#include "common.h"

#include <stdarg.h>

#include <mutex>
#include <vector>

namespace drsa {
static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

const char* last_error() { return g_err; }

namespace {
struct AttrKey {
  int dev;
  const void* fn;
  size_t bytes;
};
std::mutex g_attr_mu;
std::vector<AttrKey> g_attr_done;
constexpr int kMaxDev = 64;
int g_cus[kMaxDev] = {0};
std::mutex g_cu_mu;
}  // namespace

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  return dev;
}

int ensure_smem(const void* fn, size_t bytes) {
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_attr_mu);
  for (const AttrKey& k : g_attr_done)
    if (k.dev == dev && k.fn == fn && k.bytes >= bytes) return DRSA_OK;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) {
    set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize=%zu) on device %d: %s", bytes, dev,
              hipGetErrorString(e));
    return (int)e;
  }
  g_attr_done.push_back({dev, fn, bytes});
  return DRSA_OK;
}

int cu_count() {
  const int dev = current_device();
  if (dev >= kMaxDev) return 256;
  std::lock_guard<std::mutex> lk(g_cu_mu);
  if (!g_cus[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    g_cus[dev] = cus;
  }
  return g_cus[dev];
}
}  // namespace drsa

extern "C" const char* drsa_amd_last_error(void) { return drsa::last_error(); }
extern "C" int drsa_amd_version(void) { return 2; }
