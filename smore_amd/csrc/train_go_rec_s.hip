// go_rec_kernel instantiations (go_rec.h): MODE_STORE scatter, KMAX 5 and 10; the Go walk-pair kernel
#include "go_rec.h"
#include "go_walks.h"
SMORE_GO_REC_INST(s, smore::MODE_STORE)
SMORE_GO_PAIR_INST(s, smore::MODE_STORE)
