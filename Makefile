# libpcx.so: the MI355X (gfx950) kernels behind the C ABI in include/pcx.h.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Iinclude -Wall -Wno-unused-result \
           -munsafe-fp-atomics
SRC = $(wildcard phoneme_contrast_amd/csrc/*.hip)
OBJ = $(patsubst phoneme_contrast_amd/csrc/%.hip,build/%.o,$(SRC))
HDR = $(wildcard phoneme_contrast_amd/csrc/*.h) include/pcx.h
LIB = phoneme_contrast_amd/libpcx.so

TOOLS = tools/wino_bench tools/ww_bench tools/stem_bench tools/wb_bench

all: $(LIB) $(TOOLS)

# engine cross-check / micro-benchmark (tests/test_wino_engine_gpu.py runs it)
tools/wino_bench: tools/wino_bench.cpp $(LIB) $(HDR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude $< -Lphoneme_contrast_amd -lpcx \
	    -Wl,-rpath,'$$ORIGIN/../phoneme_contrast_amd' -o $@

# Winograd weight gradient vs the pixel-stream kernel (tests/test_wino_engine_gpu.py runs it)
tools/ww_bench: tools/ww_bench.cpp $(LIB) $(HDR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude $< -Lphoneme_contrast_amd -lpcx \
	    -Wl,-rpath,'$$ORIGIN/../phoneme_contrast_amd' -o $@

# fused layer-2 backward (wgbd_wino) vs the two-kernel path (tests/test_wino_engine_gpu.py runs it)
tools/wb_bench: tools/wb_bench.cpp $(LIB) $(HDR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude $< -Lphoneme_contrast_amd -lpcx \
	    -Wl,-rpath,'$$ORIGIN/../phoneme_contrast_amd' -o $@

# fused bf16 stem (y0 recomputed) vs the kernels that keep the y0 plane (tools/run_stem.sh runs it)
tools/stem_bench: tools/stem_bench.cpp $(LIB) $(HDR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude $< -Lphoneme_contrast_amd -lpcx \
	    -Wl,-rpath,'$$ORIGIN/../phoneme_contrast_amd' -o $@

build/%.o: phoneme_contrast_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

# fp32 MFMA shares the vector pipe: packed f32 VALU (SLP) costs more issue than scalar beside it
build/conv_wino.o: CXXFLAGS += -fno-slp-vectorize
build/wgrad_wino.o: CXXFLAGS += -fno-slp-vectorize
build/wgbd_wino.o: CXXFLAGS += -fno-slp-vectorize

$(LIB): $(OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

clean:
	rm -rf build $(LIB) $(TOOLS)

.PHONY: all clean
