// 256-thread paired gradient launches with a 128x128 data-gradient tile (see bwd_pair.h)
#include "bwd_pair.h"

CDP_PAIR_TU(128, 128)
