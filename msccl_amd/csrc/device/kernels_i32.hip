#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_i32, int32_t) }
