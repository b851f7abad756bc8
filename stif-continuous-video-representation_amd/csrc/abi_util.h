// Error reporting shared by the C-ABI entry points (thread-local last error).
#pragma once
#include <hip/hip_runtime.h>

int stif_fail(int code, const char* msg);
int stif_check_launch(const char* where);
// compute units of the current device (cached; 256 if the query fails) -- persistent-grid sizing
int stif_num_cus();
