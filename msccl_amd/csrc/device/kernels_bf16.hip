#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE_FP(gLaunch_bf16, Bf16) }
