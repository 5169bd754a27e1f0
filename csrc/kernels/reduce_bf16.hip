// K1 + IPC reductions instantiated for BF16 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(BF16, PDCC_OPS_FLOAT)
