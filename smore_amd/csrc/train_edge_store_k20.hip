// edge_train_kernel instantiations: store scatter, up to 20 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_EDGE_INST(s20, 20, smore::MODE_STORE)
