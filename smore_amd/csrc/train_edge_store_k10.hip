// edge_train_kernel instantiations: store scatter, up to 10 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_EDGE_INST(s10, 10, smore::MODE_STORE)
