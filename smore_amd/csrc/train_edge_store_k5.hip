// edge_train_kernel instantiations: store scatter, up to 5 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_EDGE_INST(s5, 5, smore::MODE_STORE)
