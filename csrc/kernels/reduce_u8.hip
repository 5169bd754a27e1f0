// K1 + IPC reductions instantiated for U8 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(U8, PDCC_OPS_INT)
