# Builds the gfx950 C-ABI library ddsp_pytorch_amd/lib/libddsp_hip.so (hipcc cross-compiles
# without a GPU).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := ddsp_pytorch_amd/csrc/synth.hip ddsp_pytorch_amd/csrc/noise.hip ddsp_pytorch_amd/csrc/reverb.hip \
       ddsp_pytorch_amd/csrc/upols.hip ddsp_pytorch_amd/csrc/synth_frame.hip \
       ddsp_pytorch_amd/csrc/backward.hip ddsp_pytorch_amd/csrc/stft.hip \
       ddsp_pytorch_amd/csrc/gru.hip ddsp_pytorch_amd/csrc/dense.hip ddsp_pytorch_amd/csrc/stream.hip
HDR := include/ddsp_hip.h ddsp_pytorch_amd/csrc/common.h ddsp_pytorch_amd/csrc/upols.h ddsp_pytorch_amd/csrc/fft_radix.h \
       ddsp_pytorch_amd/csrc/noise_dsp.h
LIB := ddsp_pytorch_amd/lib/libddsp_hip.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ibuild -Wall -Wno-unused-result
# packed-fp32 SLP vectorisation measured 10% slower on the oscillator loop (VALU-bound)
HIPFLAGS_synth := -fno-slp-vectorize
HIPFLAGS_synth_frame := -fno-slp-vectorize
HIPFLAGS_backward := -fno-slp-vectorize
# packed f32 VALU beside MFMAs costs more than the scalar pair (MI355X_MICROARCH.md cycle constants)
HIPFLAGS_dense := -fno-slp-vectorize
OBJ := $(patsubst ddsp_pytorch_amd/csrc/%.hip,build/%.o,$(SRC))

TORCH_DIR := $(shell python3 -c "import torch,os;print(os.path.dirname(torch.__file__))" 2>/dev/null)
TORCH_LIB := ddsp_pytorch_amd/lib/libddsp_hip_torch.so

RT_HOST := tools/realtime_host

all: $(LIB) $(TORCH_LIB) $(RT_HOST)

build/twiddle4096.inc: tools/gen_twiddles.py
	@mkdir -p build
	python3 tools/gen_twiddles.py 4096 > $@

build/upols.o build/noise.o build/synth_frame.o build/backward.o build/stft.o: build/twiddle4096.inc

build/%.o: ddsp_pytorch_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(HIPFLAGS_$*) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p ddsp_pytorch_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ)

# TorchScript operators torch.ops.ddsp_hip.* (host C++ over the C-ABI; no device code)
$(TORCH_LIB): ddsp_pytorch_amd/csrc/torch_ops.cpp include/ddsp_hip.h $(LIB)
	g++ -O2 -std=c++17 -shared -fPIC -o $@ $< -Iinclude -I$(TORCH_DIR)/include \
	  -I$(TORCH_DIR)/include/torch/csrc/api/include -I/opt/rocm/include -D__HIP_PLATFORM_AMD__=1 \
	  -DUSE_ROCM=1 -D_GLIBCXX_USE_CXX11_ABI=1 -L$(TORCH_DIR)/lib -lc10 -lc10_hip -ltorch -ltorch_cpu \
	  -ltorch_hip -Lddsp_pytorch_amd/lib -lddsp_hip -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(TORCH_DIR)/lib

# C++ libtorch realtime host mirroring the ddsp~ external (config 3 latency)
$(RT_HOST): tools/realtime_host.cpp
	g++ -O2 -std=c++17 $< -o $@ -I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include \
	  -D_GLIBCXX_USE_CXX11_ABI=1 -L$(TORCH_DIR)/lib -ltorch -ltorch_cpu -lc10 -Wl,--no-as-needed \
	  -ltorch_hip -Wl,--as-needed -Wl,-rpath,$(TORCH_DIR)/lib -ldl -lpthread

clean:
	rm -rf build $(LIB) $(TORCH_LIB) $(RT_HOST)

.PHONY: all clean
