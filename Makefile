# Build of the MI355X (gfx950) hot path.  No cmake: plain make + hipcc.
#   make            -> smore_amd/lib/libsmore_hip.so + smore_amd/bin/{line,bpr,mf,deepwalk}
#   make oracle     -> oracle/build/liboracle.so (test infrastructure)
#   make ref        -> oracle/_ref/ref_harness (needs /root/reference)
#   tuning variants: make lib OBJ=build/obj_x LIB=build/x/libsmore_hip.so EXTRA=-DSMORE_WAVES_HYBRID=5
#   (load one with SMORE_LIB=build/x/libsmore_hip.so)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS := -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function
EXTRA    ?=
HIPFLAGS := $(CXXFLAGS) --offload-arch=$(ARCH) -Wno-pass-failed $(EXTRA)
SRC      := smore_amd/csrc
OBJ      ?= build/obj
LIB      ?= smore_amd/lib/libsmore_hip.so
BIN      := smore_amd/bin
# kernels depend on the device headers only; host objects on the host headers
DEV_HDRS := $(SRC)/device_common.h $(SRC)/train_kernels.h $(SRC)/edge_kernels.h $(SRC)/edge_inst.h
HOST_HDRS := $(SRC)/host_graph.h $(SRC)/ctx.h $(SRC)/train_kernels.h $(SRC)/device_common.h $(SRC)/go_walks.h \
             $(SRC)/hot_exchange.h $(SRC)/comm_watch.h include/smore_hip.h

.PHONY: all lib cli goshape oracle ref clean
all: lib cli goshape

lib: $(LIB)

HOST_SRCS := host_graph loader capi exchange graphgen blocks
$(OBJ)/%.o: $(SRC)/%.cpp $(HOST_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(CXXFLAGS) -c -o $@ $<

$(OBJ)/%.o: $(SRC)/%.hip $(DEV_HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# the Go walk kernels also depend on the CTDNE declarations; the Go record
# kernels on go_rec.h; the exchange passes on their declarations
$(OBJ)/train_go.o: $(SRC)/go_walks.h
$(OBJ)/train_go_rec_s.o $(OBJ)/train_go_rec_a.o $(OBJ)/train_go_rec_h.o: $(SRC)/go_rec.h $(SRC)/go_walks.h
$(OBJ)/replica_sync.o: $(SRC)/hot_exchange.h

LIB_OBJS := $(patsubst %,$(OBJ)/%.o,$(HOST_SRCS)) $(patsubst $(SRC)/%.hip,$(OBJ)/%.o,$(wildcard $(SRC)/*.hip))

$(LIB): $(LIB_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ -lpthread -ldl

CLIS := $(patsubst $(SRC)/cli/%.cpp,$(BIN)/%,$(wildcard $(SRC)/cli/*.cpp))
cli: $(CLIS)

$(BIN)/%: $(SRC)/cli/%.cpp $(SRC)/cli/cli_common.h $(LIB)
	@mkdir -p $(BIN)
	g++ -std=c++17 -O2 -Wall -Iinclude -o $@ $< -L$(dir $(LIB)) -lsmore_hip -Wl,-rpath,'$$ORIGIN/../lib'

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

clean:
	rm -rf build smore_amd/lib smore_amd/bin

# the Go shim's call sequence as a C program (tests/test_gpu_goshape.py), and
# the Go UpdatePairs hook under concurrent callers (tests/test_gpu_pairs.py)
goshape: tests/c/go_shape tests/c/pairs_mt
tests/c/go_shape: tests/c/go_shape.c include/smore_hip.h $(LIB)
	gcc -std=c11 -O2 -Wall -Iinclude -o $@ $< -L$(dir $(LIB)) -lsmore_hip -Wl,-rpath,'$$ORIGIN/../../smore_amd/lib'
tests/c/pairs_mt: tests/c/pairs_mt.c include/smore_hip.h $(LIB)
	gcc -std=gnu11 -O2 -Wall -Iinclude -o $@ $< -L$(dir $(LIB)) -lsmore_hip -lpthread -Wl,-rpath,'$$ORIGIN/../../smore_amd/lib'
