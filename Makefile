# Build of the MI355X (gfx950) scoring backend and of the CPU oracle.
#   make            -> hhfm_amd/lib/libhhfm.so   (C ABI, HIP kernels; include/hhfm.h)
#                      hhfm_amd/lib/_hhfm*.so    (thin pybind11 binding of that ABI)
#                      oracle/liboracle.so       (C restatement used as checker / CPU baseline)
# hipcc cross-compiles gfx950 without a GPU; built .so files are git-ignored
# but travel to the GPU box with the gpurun snapshot.
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
ARCH     ?= gfx950
PYTHON   ?= python3
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
CXXFLAGS ?= -O2 -std=c++17 -fPIC -Wall

LIBDIR   := hhfm_amd/lib
CSRC     := hhfm_amd/csrc
HIP_SRCS := $(wildcard $(CSRC)/*.hip)
CPP_SRCS := $(filter-out $(CSRC)/pybind_hhfm.cpp,$(wildcard $(CSRC)/*.cpp))
OBJS     := $(patsubst $(CSRC)/%.hip,build/%.o,$(HIP_SRCS)) \
            $(patsubst $(CSRC)/%.cpp,build/%.o,$(CPP_SRCS))
LIB      := $(LIBDIR)/libhhfm.so
EXT      := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYMOD    := $(LIBDIR)/_hhfm$(EXT)
PYINC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PBINC    := $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
ORACLE   := oracle/liboracle.so

.PHONY: all clean native oracle
all: native oracle
native: $(LIB) $(PYMOD)
oracle: $(ORACLE)

build/%.o: $(CSRC)/%.hip $(wildcard $(CSRC)/*.h) include/hhfm.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/%.o: $(CSRC)/%.cpp include/hhfm.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

$(PYMOD): $(CSRC)/pybind_hhfm.cpp $(LIB) include/hhfm.h
	$(CXX) $(CXXFLAGS) -shared -I$(PYINC) -I$(PBINC) -Iinclude $< \
	  -L$(LIBDIR) -lhhfm -Wl,-rpath,'$$ORIGIN' -o $@

$(ORACLE): oracle/cpu_oracle.c
	$(CC) -O3 -march=x86-64-v2 -fopenmp -fPIC -shared -o $@ $< -lm

clean:
	rm -rf build $(LIBDIR)/*.so $(ORACLE)
