# m2dec_amd build: host parser (C) + gfx950 HIP reconstruction back end -> libm2dec_amd.so
# oracle/ (CPU restatement, test infrastructure only) -> oracle/_build/liboracle.so
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
JOBS ?= 8

INC := -Iinclude -Im2dec_amd/csrc/host
CFLAGS := -O3 -g -fPIC -Wall -Wextra -Wno-unused-parameter -std=gnu11 $(INC)
HIPFLAGS := --offload-arch=$(ARCH) -O3 -g -fPIC -std=c++17 $(INC) -Wno-unused-result

HOST_SRC := $(wildcard m2dec_amd/csrc/host/*.c)
HOST_OBJ := $(patsubst m2dec_amd/csrc/host/%.c,build/host/%.o,$(HOST_SRC))
HIP_SRC := m2dec_amd/csrc/hip/recon_hip.hip
HIP_OBJ := build/hip/recon_hip.o

LIB := m2dec_amd/lib/libm2dec_amd.so
ORACLE := oracle/_build/liboracle.so
GEN := tools/_build/h264gen

all: $(LIB) $(ORACLE) $(GEN)

build/host/%.o: m2dec_amd/csrc/host/%.c $(wildcard m2dec_amd/csrc/host/*.h) $(wildcard include/*.h)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(HIP_OBJ): $(HIP_SRC) m2dec_amd/csrc/hip/recon_kernels.h $(wildcard include/*.h)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJ) $(HIP_OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-soname,libm2dec_amd.so

$(ORACLE): oracle/recon_oracle.c include/m2d_recon.h include/m2d.h
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -fPIC -Wall -std=gnu11 -Iinclude -shared -o $@ oracle/recon_oracle.c

$(GEN): $(wildcard tools/h264gen/*.c) $(wildcard tools/h264gen/*.h) m2dec_amd/csrc/host/h264_spec_tables.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -Wall -std=gnu11 $(INC) -o $@ $(wildcard tools/h264gen/*.c) m2dec_amd/csrc/host/h264_spec_tables.c -lm

clean:
	rm -rf build m2dec_amd/lib oracle/_build tools/_build

.PHONY: all clean
