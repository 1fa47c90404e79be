# Native build: host C++ (g++) + HIP/CDNA4 kernels (hipcc, gfx950) -> one shared library plus the
# worker_node / gateway / loadgen binaries.  `make -j8` here; the artefacts travel to the GPU box.
PKG      := distributed-inference-engine-cpp_amd
SRC      := $(PKG)/csrc
BUILD    := build
ROCM     ?= /opt/rocm
ARCH     ?= gfx950
CXX      := g++
HIPCC    := $(ROCM)/bin/hipcc
LIBDIR   := $(PKG)/lib
BINDIR   := $(PKG)/bin

CXXFLAGS := -std=c++17 -O3 -march=x86-64-v3 -fPIC -fopenmp -g -Wall -Wextra -Wno-unused-parameter \
            -I$(ROCM)/include -D__HIP_PLATFORM_AMD__
HIPFLAGS := -std=c++17 -O3 --offload-arch=$(ARCH) -fPIC -g -Wall -Wno-unused-parameter -Wno-unused-result \
            -munsafe-fp-atomics
LDLIBS   := -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -lgomp -lpthread

HOST_SRCS := core/json.cpp core/http.cpp core/http_async.cpp core/log.cpp core/metrics.cpp core/shm_arena.cpp core/textpack.cpp parallel/dp_group.cpp parallel/comm.cpp engine/dp_engine.cpp serve/consistent_hash.cpp serve/circuit_breaker.cpp \
             serve/worker.cpp serve/gateway.cpp serve/loadgen.cpp onnx/onnx_model.cpp \
             engine/engine.cpp engine/cpu_exec.cpp engine/hybrid_engine.cpp engine/hip_plan.cpp capi/capi.cpp capi/capi_kernels.cpp
HIP_SRCS  := $(notdir $(wildcard $(SRC)/engine/*.hip)) $(notdir $(wildcard $(SRC)/kernels/*.hip))
HOST_OBJS := $(addprefix $(BUILD)/host/,$(HOST_SRCS:.cpp=.o))
HIP_OBJS  := $(patsubst %.hip,$(BUILD)/hip/%.o,$(HIP_SRCS))
APPS      := worker_node gateway loadgen

all: $(LIBDIR)/libdie.so $(addprefix $(BINDIR)/,$(APPS))

$(BUILD)/host/%.o: $(SRC)/%.cpp $(wildcard $(SRC)/*/*.h)
	@mkdir -p $(dir $@)
	$(CXX) $(CXXFLAGS) -MMD -c $< -o $@

$(BUILD)/hip/%.o: $(SRC)/engine/%.hip $(wildcard $(SRC)/*/*.h) $(wildcard $(SRC)/kernels/*.h)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/hip/%.o: $(SRC)/kernels/%.hip $(wildcard $(SRC)/kernels/*.h)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libdie.so: $(HOST_OBJS) $(HIP_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^ $(LDLIBS)

$(BINDIR)/%: $(SRC)/apps/%_main.cpp $(LIBDIR)/libdie.so
	@mkdir -p $(BINDIR)
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(LIBDIR) -Wl,-rpath,'$$ORIGIN/../lib' -ldie $(LDLIBS)

$(BINDIR)/worker_node: $(SRC)/apps/worker_main.cpp $(LIBDIR)/libdie.so
	@mkdir -p $(BINDIR)
	$(CXX) $(CXXFLAGS) $< -o $@ -L$(LIBDIR) -Wl,-rpath,'$$ORIGIN/../lib' -ldie $(LDLIBS)

clean:
	rm -rf $(BUILD) $(LIBDIR) $(BINDIR)

# Host-runtime concurrency stress under sanitizers; no GPU code is linked.
STRESS_SRCS := core/json.cpp core/http.cpp core/http_async.cpp core/log.cpp core/metrics.cpp core/shm_arena.cpp serve/consistent_hash.cpp serve/circuit_breaker.cpp \
               serve/gateway.cpp tests/stress_main.cpp
SANFLAGS := -std=c++17 -O1 -g -march=x86-64-v3 -fno-omit-frame-pointer -Wall -Wno-unused-parameter
stress-tsan: $(BINDIR)/die_stress_tsan
stress-asan: $(BINDIR)/die_stress_asan
$(BINDIR)/die_stress_tsan: $(addprefix $(SRC)/,$(STRESS_SRCS)) $(wildcard $(SRC)/*/*.h)
	@mkdir -p $(BINDIR)
	$(CXX) $(SANFLAGS) -fsanitize=thread $(addprefix $(SRC)/,$(STRESS_SRCS)) -o $@ -lpthread
$(BINDIR)/die_stress_asan: $(addprefix $(SRC)/,$(STRESS_SRCS)) $(wildcard $(SRC)/*/*.h)
	@mkdir -p $(BINDIR)
	$(CXX) $(SANFLAGS) -fsanitize=address,undefined -fno-sanitize-recover=undefined $(addprefix $(SRC)/,$(STRESS_SRCS)) -o $@ -lpthread

.PHONY: all clean stress-tsan stress-asan
-include $(HOST_OBJS:.o=.d)
