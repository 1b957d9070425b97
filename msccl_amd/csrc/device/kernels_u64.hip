#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_u64, uint64_t) }
