// K1 + IPC reductions instantiated for F64 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(F64, PDCC_OPS_FLOAT)
