// pair_train_kernel instantiations: hybrid scatter, up to 10 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_PAIR_INST(h10, 10, smore::MODE_HYBRID)
