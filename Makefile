# Builds the gfx950 C-ABI library ddsp_pytorch_amd/lib/libddsp_hip.so (hipcc cross-compiles
# without a GPU) and the C oracle used by tests.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := ddsp_pytorch_amd/csrc/synth.hip ddsp_pytorch_amd/csrc/noise.hip ddsp_pytorch_amd/csrc/reverb.hip
HDR := include/ddsp_hip.h ddsp_pytorch_amd/csrc/common.h
LIB := ddsp_pytorch_amd/lib/libddsp_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Wall \
            -Wno-unused-result -munsafe-fp-atomics
OBJ := $(patsubst ddsp_pytorch_amd/csrc/%.hip,build/%.o,$(SRC))

all: $(LIB)

build/%.o: ddsp_pytorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p ddsp_pytorch_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) -L/opt/rocm/lib -lrocfft -Wl,-rpath,/opt/rocm/lib

clean:
	rm -rf build $(LIB)

.PHONY: all clean
