// pair_train_kernel instantiations: plain-store scatter, up to 10 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_PAIR_INST(s10, 10, smore::MODE_STORE)
