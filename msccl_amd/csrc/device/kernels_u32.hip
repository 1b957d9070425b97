#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_u32, uint32_t) }
