// pair_train_kernel instantiations: hybrid scatter, up to 5 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_PAIR_INST(h5, 5, smore::MODE_HYBRID)
