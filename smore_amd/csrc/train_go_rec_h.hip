// go_rec_kernel instantiations (go_rec.h): MODE_HYBRID scatter, KMAX 5 and 10
#include "go_rec.h"
SMORE_GO_REC_INST(h, smore::MODE_HYBRID)
