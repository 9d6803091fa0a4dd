# Builds every native artefact in-tree (they travel to the GPU box with the snapshot).
#   blt_amd/libblt_bpe.so    product: HIP kernels for gfx950 + C ABI host library + pipeline
#   blt_amd/libblt_synth.so  seeded synthetic workloads (bench / tests)
#   blt_amd/blt              CLI drop-in for the reference `blt` binary
#   oracle/liboracle.so      CPU restatement of the reference (test infrastructure only)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CC ?= gcc

LIB := blt_amd/libblt_bpe.so
SYNTH := blt_amd/libblt_synth.so
ORACLE := oracle/liboracle.so
CLI := blt_amd/blt
OBJDIR := build

all: $(LIB) $(SYNTH) $(ORACLE) $(CLI)

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/bpe_kernels.o: blt_amd/csrc/bpe_kernels.hip blt_amd/csrc/bpe_kernels.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/blt_host.o: blt_amd/csrc/blt_host.cpp blt_amd/csrc/bpe_kernels.h include/blt_bpe.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/blt_pipeline.o: blt_amd/csrc/blt_pipeline.cpp include/blt_bpe.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJDIR)/bpe_kernels.o $(OBJDIR)/blt_host.o $(OBJDIR)/blt_pipeline.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^ -lpthread

# the `blt` command line (src/main.rs drop-in), linked against the library next to it
$(CLI): blt_amd/csrc/blt_cli.cpp include/blt_bpe.h $(LIB)
	$(CXX) -O2 -std=c++17 -Wall -pthread -o $@ $< -Lblt_amd -lblt_bpe -Wl,-rpath,'$$ORIGIN'

$(SYNTH): blt_amd/csrc/synth.c
	$(CC) -O2 -fPIC -fopenmp -shared -o $@ $<

$(ORACLE): oracle/bpe_oracle.c
	$(MAKE) -C oracle liboracle.so

clean:
	rm -rf $(OBJDIR) $(LIB) $(SYNTH) $(ORACLE) $(CLI)

.PHONY: all clean

# The timing build of the product kernel (per-wave phase stamps; tools/tile_timing.py with
# BLT_LIB_PATH=build/xp/libblt_bpe_timing.so).  Experiment variants: tools/build_variant.sh.
timing:
	bash tools/build_variant.sh timing -DBLT_TIMING
.PHONY: timing

# Host-sanitizer build (test infrastructure): the library's host code with ASan and
# UBSan (device code untouched), linked into tests/native/sanitize_driver.cpp with the C oracle as
# the checker.  `build/san/blt_sanitize_driver --cpu` runs the host-only checks (no GPU needed).
SANFLAGS := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
            -Xarch_host -fno-sanitize-recover=undefined
SAN := build/san
# one compiler for every instrumented object (one sanitizer runtime)
SANCC := /opt/rocm/lib/llvm/bin/clang
sanitize: $(SAN)/blt_sanitize_driver
$(SAN):
	mkdir -p $(SAN)
$(SAN)/blt_host.o: blt_amd/csrc/blt_host.cpp blt_amd/csrc/bpe_kernels.h include/blt_bpe.h | $(SAN)
	$(HIPCC) $(HIPFLAGS) -O1 $(SANFLAGS) -x hip -c $< -o $@
$(SAN)/blt_pipeline.o: blt_amd/csrc/blt_pipeline.cpp include/blt_bpe.h | $(SAN)
	$(HIPCC) $(HIPFLAGS) -O1 $(SANFLAGS) -x hip -c $< -o $@
$(SAN)/oracle.o: oracle/bpe_oracle.c | $(SAN)
	$(SANCC) -O1 -g -fPIC -std=c11 -pthread -fsanitize=address,undefined -fno-omit-frame-pointer -c $< -o $@
$(SAN)/driver.o: tests/native/sanitize_driver.cpp include/blt_bpe.h | $(SAN)
	$(SANCC)++ -O1 -g -std=c++17 -pthread -fsanitize=address,undefined -fno-omit-frame-pointer -c $< -o $@
$(SAN)/blt_sanitize_driver: $(SAN)/driver.o $(OBJDIR)/bpe_kernels.o $(SAN)/blt_host.o $(SAN)/blt_pipeline.o $(SAN)/oracle.o
	$(HIPCC) -fno-gpu-sanitize -fsanitize=address,undefined -o $@ $^ -lpthread
.PHONY: sanitize
