# bedops_amd build: libbedgpu (HIP, gfx950) + C front-ends + tools + CPU oracle.
# Everything is built in-tree so the artefacts travel to the GPU box with the repo.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CC ?= gcc
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -Wall -Wno-unused-value -Wno-unused-result
CFLAGS ?= -O2 -std=gnu11 -pthread -Wall -Wno-unused-result

SRC := bedops_amd/csrc
OBJ := build/obj
LIB := bedops_amd/lib/libbedgpu.so
BIN := bedops_amd/bin
HIPSRCS := $(wildcard $(SRC)/*.hip)
HIPOBJS := $(patsubst $(SRC)/%.hip,$(OBJ)/%.o,$(HIPSRCS))
CLIS := $(BIN)/bedops $(BIN)/bedmap $(BIN)/closest-features $(BIN)/sort-bed

all: lib cli tools oracle

lib: $(LIB)
cli: $(CLIS)
tools: tools/build/libbedgen.so tools/build/bedgen tools/build/heap_replay_check

$(OBJ)/%.o: $(SRC)/%.hip $(wildcard $(SRC)/*.h) include/bedgpu.h
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# bg_build_hash(): content hash of the sources, Makefile and flags (tools/src_hash.py), checked
# by tests/conftest.py against the tree; the file is rewritten only when the hash changes
BUILD_FLAGS = $(HIPFLAGS) ARCH=$(ARCH)
$(OBJ)/bg_buildhash.c: FORCE
	@mkdir -p $(OBJ)
	@python3 tools/src_hash.py --flags "$(BUILD_FLAGS)" --write $@ > /dev/null

$(OBJ)/bg_buildhash.o: $(OBJ)/bg_buildhash.c
	$(CC) -O2 -fPIC -c $< -o $@

$(LIB): $(HIPOBJS) $(OBJ)/bg_buildhash.o
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ -L/opt/rocm/lib -lz -ldl -Wl,-rpath,/opt/rocm/lib

print-hash:
	@python3 tools/src_hash.py --flags "$(BUILD_FLAGS)"

$(BIN)/%: bedops_amd/cli/%.c bedops_amd/cli/cli_common.h bedops_amd/cli/cli_shard.h bedops_amd/cli/cli_stream.h include/bedgpu.h $(LIB)
	@mkdir -p $(BIN)
	$(CC) $(CFLAGS) -o $@ $< -Lbedops_amd/lib -lbedgpu -Wl,-rpath,'$$ORIGIN/../lib' -Wl,-rpath,/opt/rocm/lib

$(BIN)/sort-bed: bedops_amd/cli/sortbed.c bedops_amd/cli/cli_common.h include/bedgpu.h $(LIB)
	@mkdir -p $(BIN)
	$(CC) $(CFLAGS) -o $@ $< -Lbedops_amd/lib -lbedgpu -Wl,-rpath,'$$ORIGIN/../lib' -Wl,-rpath,/opt/rocm/lib

$(BIN)/closest-features: bedops_amd/cli/closest.c bedops_amd/cli/cli_common.h bedops_amd/cli/cli_shard.h bedops_amd/cli/cli_stream.h include/bedgpu.h $(LIB)
	@mkdir -p $(BIN)
	$(CC) $(CFLAGS) -o $@ $< -Lbedops_amd/lib -lbedgpu -Wl,-rpath,'$$ORIGIN/../lib' -Wl,-rpath,/opt/rocm/lib

tools/build/libbedgen.so: tools/bedgen.c
	@mkdir -p tools/build
	$(CC) -O3 -fopenmp -shared -fPIC -o $@ $<

tools/build/bedgen: tools/bedgen.c
	@mkdir -p tools/build
	$(CC) -O3 -fopenmp -DBEDGEN_MAIN -o $@ $<

# the host heap replay (bg_heap_replay.h) on the CPU, checked against the oracle's addresses
tools/build/heap_replay_check: tools/heap_replay_check.cpp $(SRC)/bg_heap_replay.h $(SRC)/bg_internal.h include/bedgpu.h
	@mkdir -p tools/build
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -o $@ $<

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build bedops_amd/lib bedops_amd/bin tools/build
	$(MAKE) -C oracle clean

.PHONY: all lib cli tools oracle clean print-hash FORCE
FORCE:
