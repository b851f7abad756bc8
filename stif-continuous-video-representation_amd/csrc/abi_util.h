// Error reporting shared by the C-ABI entry points (thread-local last error).
#pragma once
#include <hip/hip_runtime.h>

int stif_fail(int code, const char* msg);
int stif_check_launch(const char* where);
