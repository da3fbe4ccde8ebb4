# Builds the C-ABI library (gfx950 only) in-tree: vaeunet_amd/libvaeunet_hip.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
SRC   := $(wildcard vaeunet_amd/csrc/*.hip)
OBJ   := $(patsubst vaeunet_amd/csrc/%.hip,build/%.o,$(SRC))
LIB   := vaeunet_amd/libvaeunet_hip.so
FLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-pass-failed

all: $(LIB)

build/%.o: vaeunet_amd/csrc/%.hip vaeunet_amd/csrc/common.h include/vaeunet.h
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

oracle: oracle/_ref
oracle/_ref:
	@mkdir -p oracle/_ref

clean:
	rm -rf build $(LIB)

.PHONY: all clean oracle
