// 256-thread paired gradient launches with a 64x64 data-gradient tile (see bwd_pair.h)
#include "bwd_pair.h"

CDP_PAIR_TU(64, 64)
