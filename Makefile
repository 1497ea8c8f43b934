# m2dec_amd build: host parser (C) + gfx950 HIP reconstruction back end -> libm2dec_amd.so
# oracle/ (CPU restatement, test infrastructure only) -> oracle/_build/liboracle.so
HIPCC ?= /opt/rocm/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
JOBS ?= 8

INC := -Iinclude -Im2dec_amd/csrc/host
# host code: x86-64-v3 (AVX2 / BMI2 / LZCNT: every MI355X host CPU, EPYC Zen 4/5) — ~9 % faster CABAC parse
HOST_ARCH ?= -march=x86-64-v3
CFLAGS := -O3 -g -fPIC $(HOST_ARCH) -Wall -Wextra -Wno-unused-parameter -std=gnu11 $(INC)
HIPFLAGS := --offload-arch=$(ARCH) -O3 -g -fPIC -std=c++17 $(INC) -Wno-unused-result

HOST_SRC := $(wildcard m2dec_amd/csrc/host/*.c)
HOST_OBJ := $(patsubst m2dec_amd/csrc/host/%.c,build/host/%.o,$(HOST_SRC))
HIP_SRC := m2dec_amd/csrc/hip/recon_hip.hip
HIP_HDR := m2dec_amd/csrc/hip/h265_mfma.h m2dec_amd/csrc/hip/selftest_data.h m2dec_amd/csrc/hip/recon_kernels.h m2dec_amd/csrc/hip/recon_internal.h m2dec_amd/csrc/host/h265_dec.h
HIP_OBJ := build/hip/recon_hip.o build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o

LIB := m2dec_amd/lib/libm2dec_amd.so
ORACLE := oracle/_build/liboracle.so
GEN := tools/_build/h264gen
GEN265 := tools/_build/h265gen
M2VGEN := tools/_build/m2vgen

APP := m2dec_amd/lib/h264dec
HARNESS := tools/_build/m2decoder_like

MFMA_PROBE := tools/_build/mfma_idct_probe

all: $(LIB) $(ORACLE) $(GEN) $(GEN265) $(M2VGEN) $(APP) $(HARNESS) $(MFMA_PROBE)

# the H.265 int8-MFMA inverse DCT against the reference's integer transform on the GPU (tests/test_gpu_h265.py)
$(MFMA_PROBE): tools/mfma_idct_probe.hip m2dec_amd/csrc/hip/h265_mfma.h
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Im2dec_amd/csrc/hip -o $@ $<

# test harness: drives h264d_func the way src/app/m2decoder.h does (no release call)
$(HARNESS): tests/harness/m2decoder_like.cpp $(LIB) include/m2dec_amd.h include/m2d.h
	@mkdir -p $(dir $@)
	g++ -O2 -g -Wall -std=c++17 -Iinclude -o $@ $< -Lm2dec_amd/lib -lm2dec_amd -ldl -Wl,-rpath,'$$ORIGIN/../../m2dec_amd/lib'

$(APP): m2dec_amd/csrc/app/h264dec.c $(LIB) include/m2dec_amd.h
	$(CC) -O2 -Wall -std=gnu11 -Iinclude -o $@ $< -Lm2dec_amd/lib -lm2dec_amd -Wl,-rpath,'$$ORIGIN'

# the CPU guard itself must run on any x86-64: no HOST_ARCH
build/host/cpucheck.o: m2dec_amd/csrc/host/cpucheck.c
	@mkdir -p $(dir $@)
	$(CC) $(filter-out $(HOST_ARCH),$(CFLAGS)) -c $< -o $@

build/host/%.o: m2dec_amd/csrc/host/%.c $(wildcard m2dec_amd/csrc/host/*.h) $(wildcard include/*.h)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

build/hip/%.o: m2dec_amd/csrc/hip/%.hip $(HIP_HDR) $(wildcard include/*.h)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJ) $(HIP_OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-soname,libm2dec_amd.so -Wl,--no-undefined -lpthread

$(ORACLE): oracle/recon_oracle.c oracle/h265_oracle.c include/m2d_recon.h include/m2d.h
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -fPIC -Wall -std=gnu11 -Iinclude -shared -o $@ oracle/recon_oracle.c oracle/h265_oracle.c

$(GEN265): tools/h265gen/h265gen.c tools/h264gen/cabac_enc.c tools/h264gen/bitwriter.h m2dec_amd/csrc/host/h264_spec_tables.c m2dec_amd/csrc/host/h265_tables.c m2dec_amd/csrc/host/h265_dec.h
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -Wall -std=gnu11 $(INC) -o $@ tools/h265gen/h265gen.c tools/h264gen/cabac_enc.c m2dec_amd/csrc/host/h264_spec_tables.c m2dec_amd/csrc/host/h265_tables.c -lm

$(GEN): $(wildcard tools/h264gen/*.c) $(wildcard tools/h264gen/*.h) m2dec_amd/csrc/host/h264_spec_tables.c
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -Wall -std=gnu11 $(INC) -o $@ $(wildcard tools/h264gen/*.c) m2dec_amd/csrc/host/h264_spec_tables.c -lm

$(M2VGEN): tools/m2vgen/m2vgen.c m2dec_amd/csrc/host/mpeg2_tables.c m2dec_amd/csrc/host/mpeg2_dec.h tools/h264gen/bitwriter.h
	@mkdir -p $(dir $@)
	$(CC) -O2 -g -Wall -std=gnu11 $(INC) -o $@ tools/m2vgen/m2vgen.c m2dec_amd/csrc/host/mpeg2_tables.c -lm

DBG_LIB := build/dbg/libm2dec_amd_stamps.so
$(DBG_LIB): $(HOST_OBJ) $(HIP_SRC) $(HIP_HDR) build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DM2DEC_STAMPS -c $(HIP_SRC) -o build/dbg/recon_hip_stamps.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HOST_OBJ) build/dbg/recon_hip_stamps.o build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o -Wl,--no-undefined

stamps: $(DBG_LIB)

# H.265 CTU kernel stamps (tools/stamps_h265.py)
H5S_LIB := build/h5s/libm2dec_amd_h5stamps.so
$(H5S_LIB): $(HOST_OBJ) m2dec_amd/csrc/hip/h265_hip.hip $(HIP_HDR) build/hip/recon_hip.o build/hip/runtime.o build/hip/m2v_hip.o
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DH265_STAMPS -c m2dec_amd/csrc/hip/h265_hip.hip -o build/h5s/h265_hip_stamps.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HOST_OBJ) build/hip/recon_hip.o build/hip/runtime.o build/hip/m2v_hip.o build/h5s/h265_hip_stamps.o -Wl,--no-undefined

h5stamps: $(H5S_LIB)

# diagnostic variants: make variant V=NAME FLAGS="-DX"
variant: $(HOST_OBJ) build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o
	@mkdir -p build/var
	$(HIPCC) $(HIPFLAGS) $(FLAGS) -c $(HIP_SRC) -o build/var/recon_$(V).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/var/lib_$(V).so $(HOST_OBJ) build/var/recon_$(V).o build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o -Wl,--no-undefined

clean:
	rm -rf build m2dec_amd/lib oracle/_build tools/_build

.PHONY: all clean stamps variant h5stamps

# inter MB phase stamps (tools/stamps_interw.py)
STW_LIB := build/dbg/libm2dec_amd_stampw.so
$(STW_LIB): $(HOST_OBJ) $(HIP_SRC) $(HIP_HDR) build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DM2DEC_STAMPS -DM2DEC_STAMPW -DM2DEC_NO_STAMPI -c $(HIP_SRC) -o build/dbg/recon_hip_stampw.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HOST_OBJ) build/dbg/recon_hip_stampw.o build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o -Wl,--no-undefined

stampw: $(STW_LIB)

# deblocking filter sub-step stamps (tools/stamps_dbk.py)
STD_LIB := build/dbg/libm2dec_amd_stampd.so
$(STD_LIB): $(HOST_OBJ) $(HIP_SRC) $(HIP_HDR) build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DM2DEC_STAMPS -DM2DEC_STAMPD -DM2DEC_NO_STAMPI -c $(HIP_SRC) -o build/dbg/recon_hip_stampd.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(HOST_OBJ) build/dbg/recon_hip_stampd.o build/hip/runtime.o build/hip/m2v_hip.o build/hip/h265_hip.o -Wl,--no-undefined

stampd: $(STD_LIB)
