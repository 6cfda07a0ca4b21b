// go_rec_kernel instantiations (go_rec.h): MODE_HYBRID scatter, KMAX 5 and 10
#include "go_rec.h"
#include "go_walks.h"
SMORE_GO_REC_INST(h, smore::MODE_HYBRID)
SMORE_GO_PAIR_INST(h, smore::MODE_HYBRID)
