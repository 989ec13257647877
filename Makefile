# Builds music-recommendation-multimodal_amd/lib/libttmi.so (gfx950 code objects, C ABI in include/ttmi.h).
PKG      := music-recommendation-multimodal_amd
SRC      := $(wildcard $(PKG)/csrc/*.hip)
OBJ      := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRC))
LIB      := $(PKG)/lib/libttmi.so
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CXXFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude
DEPS     := $(wildcard $(PKG)/csrc/*.h) include/ttmi.h

.PHONY: all clean
all: $(LIB)

build/%.o: $(PKG)/csrc/%.hip $(DEPS)
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p $(PKG)/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

clean:
	rm -rf build $(LIB)
