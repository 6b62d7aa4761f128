# Builds the gfx950 C-ABI library ddsp_pytorch_amd/lib/libddsp_hip.so (hipcc cross-compiles
# without a GPU).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := ddsp_pytorch_amd/csrc/synth.hip ddsp_pytorch_amd/csrc/noise.hip ddsp_pytorch_amd/csrc/reverb.hip \
       ddsp_pytorch_amd/csrc/upols.hip
HDR := include/ddsp_hip.h ddsp_pytorch_amd/csrc/common.h ddsp_pytorch_amd/csrc/upols.h
LIB := ddsp_pytorch_amd/lib/libddsp_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ibuild -Wall -Wno-unused-result
# packed-fp32 SLP vectorisation measured 10% slower on the oscillator loop (VALU-bound)
HIPFLAGS_synth := -fno-slp-vectorize
OBJ := $(patsubst ddsp_pytorch_amd/csrc/%.hip,build/%.o,$(SRC))

all: $(LIB)

build/twiddle4096.inc: tools/gen_twiddles.py
	@mkdir -p build
	python3 tools/gen_twiddles.py 4096 > $@

build/upols.o build/noise.o: build/twiddle4096.inc

build/%.o: ddsp_pytorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(HIPFLAGS_$*) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p ddsp_pytorch_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
