// pair_train_kernel instantiations: atomic scatter, up to 5 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_PAIR_INST(a5, 5, smore::MODE_ATOMIC)
