// K1 + IPC reductions instantiated for I64 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(I64, PDCC_OPS_INT)
