# Builds the gfx950 kernel library retr_amd/libretr_hip.so (C-ABI declared in include/retr_hip.h)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS = -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics -Wall -Wno-unused-function
SRC_DIR = retr_amd/csrc
OBJ_DIR = build/obj
HIP_SRCS = $(wildcard $(SRC_DIR)/*.hip)
CPP_SRCS = $(wildcard $(SRC_DIR)/*.cpp)
OBJS = $(patsubst $(SRC_DIR)/%.hip,$(OBJ_DIR)/%.o,$(HIP_SRCS)) $(patsubst $(SRC_DIR)/%.cpp,$(OBJ_DIR)/%.o,$(CPP_SRCS))
HDRS = $(wildcard $(SRC_DIR)/*.hpp) include/retr_hip.h
LIB = retr_amd/libretr_hip.so

all: $(LIB)

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.cpp $(HDRS)
	@mkdir -p $(OBJ_DIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

# MFMA accumulators in VGPRs: the attention kernels' per-tile score accumulators (and the
# decode FFN's) otherwise round-trip through AGPRs (v_accvgpr_read / write: ~190 of ~1050 VALU
# per dK/dV tile); the GEMM main loops compile to the same instructions either way
$(OBJ_DIR)/attention2.o $(OBJ_DIR)/decode.o: CXXFLAGS += -mllvm -amdgpu-mfma-vgpr-form

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJS) -o $@

clean:
	rm -rf $(OBJ_DIR) $(LIB)

.PHONY: all clean
