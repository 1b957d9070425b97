#include "kernels.h"
namespace msccl { MSCCL_DEFINE_TABLE(gLaunch_f64, double) }
