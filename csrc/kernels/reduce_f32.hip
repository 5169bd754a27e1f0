// K1 + IPC reductions instantiated for F32 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(F32, PDCC_OPS_FLOAT)
