# oracle/ref.mk — build recipe for the REFERENCE ggml-cpu oracle (test infrastructure only).
#
# Compiles upstream ggml sources *where they lie* under $(REF) (read-only) with plain
# gcc/g++; every output goes to oracle/_ref/ (git-ignored; travels to the GPU box with
# the gpurun snapshot so the reference CPU path can be timed there as `cpu_baseline`).
# Nothing from the reference is copied into this repository.
#
#   make -f oracle/ref.mk            # from the repo root; needs /root/reference
#
# Products:
#   _ref/libggml-ref.so       ggml-base + ggml-cpu + registry in one library, CPU statically
#                             registered (GGML_USE_CPU), loadable-plugin support intact
#                             (GGML_BACKEND_PATH) so upstream harnesses can load our backend.
#   _ref/test-backend-ops     upstream differential harness (tests/test-backend-ops.cpp)
#   _ref/test-quantize-fns    upstream quantization pins (tests/test-quantize-fns.cpp)
#   _ref/gen_golden           our fixture generator (oracle/gen_golden.cpp) linked to the above
#   _ref/ref_cpu_bench        our CPU-baseline timer (oracle/ref_cpu_bench.cpp) linked to the above
#   _ref/gpt2_ref             GPT-2 logits / decode timing through the reference ggml graph
#                             (oracle/gpt2_ref.cpp), CPU or the reference scheduler + our plugin
#   _ref/gpt-2-sched          the reference example itself, unmodified: examples/gpt-2/main-sched.cpp
#                             + examples/common{,-ggml}.cpp (CPU backend; pins gpt2_ref's greedy stream)
#   _ref/split_check          MUL_MAT with src0 in our split (row-sharded) buffer type vs ggml-cpu,
#                             driven through the reference's backend API (oracle/split_check.cpp)
#   _ref/repack_check         MUL_MAT with src0 in our repacked-weight (extra) buffer type vs ggml-cpu
#                             (oracle/repack_check.cpp)
#   _ref/cpy_check            a seeded sweep of test-backend-ops' CPY cases, plugin vs ggml-cpu
#                             (oracle/cpy_check.cpp)
#   _ref/fusion_check         the GPT-2 node chains the plugin fuses, plugin vs ggml-cpu, through the
#                             reference's graph API and allocator (oracle/fusion_check.cpp)
#
# ISA: x86-64-v3 (AVX2/FMA/F16C) so the binaries also run on the GPU box's EPYC host;
# -march=native here could emit AVX-512/AMX the box may lack.

REF    ?= /root/reference
OUT    ?= oracle/_ref
OBJ    := $(OUT)/obj
ARCH   ?= -march=x86-64-v3
DEFS   := -DGGML_VERSION=\"ref-local\" -DGGML_COMMIT=\"ref-local\" -DGGML_SCHED_MAX_COPIES=4 \
          -D_GNU_SOURCE -D_XOPEN_SOURCE=600 -DGGML_USE_CPU -DGGML_USE_OPENMP -DGGML_USE_CPU_REPACK \
          -DNDEBUG
INCS   := -I$(REF)/include -I$(REF)/src -I$(REF)/src/ggml-cpu
# ggml-base is built WITHOUT arch flags (as upstream CMake does: only ggml-cpu gets the
# GGML_NATIVE / -march flags), so its quantizers contain no FMA contractions.
CFLAGS_BASE   := -O3 -fPIC -pthread -fopenmp -std=gnu11 $(DEFS) $(INCS) -w
CXXFLAGS_BASE := -O3 -fPIC -pthread -fopenmp -std=gnu++17 $(DEFS) $(INCS) -w
CFLAGS        := $(CFLAGS_BASE) $(ARCH)
CXXFLAGS      := $(CXXFLAGS_BASE) $(ARCH)

BASE_C   := ggml.c ggml-alloc.c ggml-quants.c
BASE_CXX := ggml.cpp ggml-backend.cpp ggml-opt.cpp ggml-threading.cpp gguf.cpp ggml-backend-reg.cpp
CPU_C    := ggml-cpu/ggml-cpu.c ggml-cpu/quants.c ggml-cpu/arch/x86/quants.c
CPU_CXX  := ggml-cpu/ggml-cpu.cpp ggml-cpu/repack.cpp ggml-cpu/hbm.cpp ggml-cpu/traits.cpp \
            ggml-cpu/binary-ops.cpp ggml-cpu/unary-ops.cpp ggml-cpu/vec.cpp ggml-cpu/ops.cpp \
            ggml-cpu/arch/x86/repack.cpp ggml-cpu/amx/amx.cpp ggml-cpu/amx/mmq.cpp

OBJS := $(patsubst %.c,$(OBJ)/%.c.o,$(BASE_C) $(CPU_C)) $(patsubst %.cpp,$(OBJ)/%.cpp.o,$(BASE_CXX) $(CPU_CXX))

all: $(OUT)/libggml-ref.so $(OUT)/test-backend-ops $(OUT)/test-quantize-fns $(OUT)/gen_golden $(OUT)/ref_cpu_bench $(OUT)/gpt2_ref \
     $(OUT)/gpt-2-sched $(OUT)/split_check $(OUT)/fusion_check $(OUT)/repack_check $(OUT)/cpy_check

$(OBJ)/ggml-cpu/%.c.o: $(REF)/src/ggml-cpu/%.c
	@mkdir -p $(dir $@)
	gcc $(CFLAGS) -c $< -o $@

$(OBJ)/ggml-cpu/%.cpp.o: $(REF)/src/ggml-cpu/%.cpp
	@mkdir -p $(dir $@)
	g++ $(CXXFLAGS) -c $< -o $@

$(OBJ)/%.c.o: $(REF)/src/%.c
	@mkdir -p $(dir $@)
	gcc $(CFLAGS_BASE) -c $< -o $@

$(OBJ)/%.cpp.o: $(REF)/src/%.cpp
	@mkdir -p $(dir $@)
	g++ $(CXXFLAGS_BASE) -c $< -o $@

$(OUT)/libggml-ref.so: $(OBJS)
	g++ -shared -fopenmp -pthread -o $@ $^ -ldl -lm

LINK := -L$(OUT) -Wl,-rpath,'$$ORIGIN' -lggml-ref -fopenmp -pthread -ldl -lm

$(OUT)/test-backend-ops: $(REF)/tests/test-backend-ops.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/test-quantize-fns: $(REF)/tests/test-quantize-fns.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/gen_golden: oracle/gen_golden.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/ref_cpu_bench: oracle/ref_cpu_bench.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/gpt2_ref: oracle/gpt2_ref.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/gpt-2-sched: $(REF)/examples/gpt-2/main-sched.cpp $(REF)/examples/common.cpp $(REF)/examples/common-ggml.cpp $(OUT)/libggml-ref.so
	g++ -O3 -pthread -std=gnu++17 -w $(ARCH) -DNDEBUG -I$(REF)/include -I$(REF)/examples $(REF)/examples/gpt-2/main-sched.cpp \
	    $(REF)/examples/common.cpp $(REF)/examples/common-ggml.cpp -o $@ $(LINK)

$(OUT)/split_check: oracle/split_check.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/fusion_check: oracle/fusion_check.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/repack_check: oracle/repack_check.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

$(OUT)/cpy_check: oracle/cpy_check.cpp $(OUT)/libggml-ref.so
	g++ $(CXXFLAGS) $< -o $@ $(LINK)

clean:
	rm -rf $(OUT)

.PHONY: all clean
