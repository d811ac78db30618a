# Builds the C-ABI HIP library (gfx950) and the C oracle pieces.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-function
SRC := $(wildcard video_style_transfer_amd/csrc/*.hip)
OBJ := $(patsubst video_style_transfer_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := video_style_transfer_amd/libvst_hip.so

all: $(LIB)

build/%.o: video_style_transfer_amd/csrc/%.hip video_style_transfer_amd/csrc/vst_common.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
