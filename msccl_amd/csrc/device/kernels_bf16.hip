#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_bf16, Bf16) }
