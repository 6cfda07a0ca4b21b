// pair_train_kernel instantiations: plain-store scatter, up to 5 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_PAIR_INST(s5, 5, smore::MODE_STORE)
