# libpcx.so: the MI355X (gfx950) kernels behind the C ABI in include/pcx.h.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# AB: compile-time A/B alternates for analysis builds only (PCX_AB_* in csrc/pcx_common.h), e.g.
#   make AB="-DPCX_AB_NO_WGBD=1" LIB=tools/ab/libpcx.so BUILD=tools/ab/obj
AB ?=
CXXFLAGS = -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Iinclude -Wall -Wno-unused-result \
           -munsafe-fp-atomics $(AB)
SRC = $(wildcard phoneme_contrast_amd/csrc/*.hip)
BUILD ?= build
OBJ = $(patsubst phoneme_contrast_amd/csrc/%.hip,$(BUILD)/%.o,$(SRC))
HDR = $(wildcard phoneme_contrast_amd/csrc/*.h) include/pcx.h
LIB ?= phoneme_contrast_amd/libpcx.so

TOOLS = tools/wino_bench tools/ww_bench tools/stem_bench tools/wb_bench tools/ws_bench

all: $(LIB) $(TOOLS)

# engine cross-check / micro-benchmark (tests/test_wino_engine_gpu.py runs it)
tools/wino_bench: tools/wino_bench.cpp $(LIB) $(HDR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude $< -Lphoneme_contrast_amd -lpcx \
	    -Wl,-rpath,'$$ORIGIN/../phoneme_contrast_amd' -o $@

# Winograd weight gradient vs the pixel-stream kernel (tests/test_wino_engine_gpu.py runs it)
tools/ww_bench: tools/ww_bench.cpp $(LIB) $(HDR)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude $< -Lphoneme_contrast_amd -lpcx \
	    -Wl,-rpath,'$$ORIGIN/../phoneme_contrast_amd' -o $@

# 32x32 row-window weight gradient (wgrad_w32) vs the pixel-stream kernel (tests/test_wino_engine_gpu.py runs it)
tools/ws_bench: tools/ws_bench.cpp $(LIB) $(HDR)
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

$(BUILD)/%.o: phoneme_contrast_amd/csrc/%.hip $(HDR)
	@mkdir -p $(BUILD)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

# fp32 MFMA shares the vector pipe: packed f32 VALU (SLP) costs more issue than scalar beside it
$(BUILD)/conv_wino.o: CXXFLAGS += -fno-slp-vectorize
$(BUILD)/wgrad_wino.o: CXXFLAGS += -fno-slp-vectorize
$(BUILD)/wgbd_wino.o: CXXFLAGS += -fno-slp-vectorize

$(LIB): $(OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

# host-side sanitizer build (no GPU): every source compiled host-only with ASan + UBSan, linked with the
# plan-builder check tools/plan_check.cpp (tests/test_plan_asan.py runs it)
ASAN_FLAGS = -O1 -g -std=c++17 --offload-arch=$(ARCH) -fPIC -Iinclude -Xarch_host -fsanitize=address \
             -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=all
ASAN_OBJ = $(patsubst phoneme_contrast_amd/csrc/%.hip,build_asan/%.o,$(SRC))

build_asan/%.o: phoneme_contrast_amd/csrc/%.hip $(HDR)
	@mkdir -p build_asan
	$(HIPCC) $(ASAN_FLAGS) -c $< -o $@

build_asan/plan_check.o: tools/plan_check.cpp include/pcx.h
	@mkdir -p build_asan
	$(HIPCC) $(ASAN_FLAGS) -c $< -o $@

tools/plan_check_asan: build_asan/plan_check.o $(ASAN_OBJ)
	$(HIPCC) -fsanitize=address,undefined build_asan/plan_check.o $(ASAN_OBJ) -o $@

asan: tools/plan_check_asan

clean:
	rm -rf build build_asan $(LIB) $(TOOLS) tools/plan_check_asan

.PHONY: all asan clean
