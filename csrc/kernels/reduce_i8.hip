// K1 + IPC reductions instantiated for I8 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(I8, PDCC_OPS_INT)
