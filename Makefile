# Builds the C-ABI HIP library (gfx950) and the C oracle pieces.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -fPIC -std=c++17 --offload-arch=$(ARCH) -Wall -Wno-unused-function
SRC := $(wildcard video_style_transfer_amd/csrc/*.hip)
OBJ := $(patsubst video_style_transfer_amd/csrc/%.hip,build/%.o,$(SRC))
LIB := video_style_transfer_amd/libvst_hip.so

all: $(LIB)

HDR := $(wildcard video_style_transfer_amd/csrc/*.h) include/vst.h

build/%.o: video_style_transfer_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJ) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
