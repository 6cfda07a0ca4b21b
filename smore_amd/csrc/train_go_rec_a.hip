// go_rec_kernel instantiations (go_rec.h): MODE_ATOMIC scatter, KMAX 5 and 10; the Go walk-pair kernel
#include "go_rec.h"
#include "go_walks.h"
SMORE_GO_REC_INST(a, smore::MODE_ATOMIC)
SMORE_GO_PAIR_INST(a, smore::MODE_ATOMIC)
