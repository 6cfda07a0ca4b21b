// edge_train_kernel instantiations: atomic scatter, up to 20 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_EDGE_INST(a20, 20, smore::MODE_ATOMIC)
