#include <stdio.h>
#include <string.h>

#include "abi_util.h"
#include "stif.h"

static thread_local char g_err[512] = "";

int stif_fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int stif_check_launch(const char* where) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", where, hipGetErrorString(e));
    return STIF_E_LAUNCH;
  }
  return STIF_OK;
}

extern "C" const char* stif_last_error(void) { return g_err; }
extern "C" const char* stif_version(void) { return "stif_hip 0.1 gfx950"; }

int stif_num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}
