// K1 + IPC reductions instantiated for F16 (see reduce_impl.h)
#include "reduce_impl.h"

PDCC_REDUCE_DTYPE(F16, PDCC_OPS_FLOAT)
