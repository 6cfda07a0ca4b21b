// pair_train_kernel instantiations: atomic scatter, up to 10 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_PAIR_INST(a10, 10, smore::MODE_ATOMIC)
