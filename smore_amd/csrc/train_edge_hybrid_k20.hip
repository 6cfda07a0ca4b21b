// edge_train_kernel instantiations: hybrid scatter, up to 20 negatives (edge_inst.h)
#include "edge_inst.h"
SMORE_EDGE_INST(h20, 20, smore::MODE_HYBRID)
