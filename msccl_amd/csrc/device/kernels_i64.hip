#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_i64, int64_t) }
