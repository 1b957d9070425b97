#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_u8, uint8_t) }
