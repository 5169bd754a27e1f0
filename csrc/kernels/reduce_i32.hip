// K1 + IPC reductions instantiated for I32 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(I32, PDCC_OPS_INT)
