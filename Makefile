# Builds the gfx950 engine (lambdafs_amd/libhrs.so) and the test-only CPU
# oracle (oracle/liboracle.so). `python -c "import __graft_entry__ as g; g.build()"`
# runs the same recipe.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CC       ?= gcc

LIB      := lambdafs_amd/libhrs.so
PROBE    := lambdafs_amd/libhrs_probe.so
ORACLE   := oracle/liboracle.so
HDRS     := Makefile include/hrs.h lambdafs_amd/csrc/hrs_device.hpp lambdafs_amd/csrc/hrs_launch.hpp lambdafs_amd/csrc/gf256.hpp lambdafs_amd/csrc/hrs_internal.hpp \
            lambdafs_amd/csrc/crc32.hpp lambdafs_amd/csrc/hrs_crc.hpp lambdafs_amd/csrc/xor_sched.hpp lambdafs_amd/csrc/hrs_codec.hpp \
            lambdafs_amd/csrc/hrs_host.hpp

# Host translation units of the C ABI (no kernels): lifecycle + queries,
# matrices, device dispatch + CRC, host-buffer path, batches.
API_SRC  := hrs_api hrs_matrix hrs_dispatch hrs_hostpath hrs_batch_api
API_OBJ  := $(patsubst %,build/%.o,$(API_SRC))

JNI      := lambdafs_amd/libhrs_jni.so
HARNESS  := tests/cpp/codec_harness tests/cpp/crc_model tests/cpp/jni_harness tests/cpp/host_logic tests/cpp/crc_tables \
            tests/cpp/copy_pool_test

TOOLS    := tools/host_call_rate tools/host_pipeline_sweep tools/host_copy_probe

all: $(LIB) $(PROBE) $(ORACLE) $(JNI) $(HARNESS) $(TOOLS)

# The synchronous C-ABI call rate (bench.py's host_calls leg, profiles/r05/).
tools/host_call_rate: tools/host_call_rate.cpp include/hrs.h $(LIB)
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ $< -Llambdafs_amd -lhrs -Wl,-rpath,'$$ORIGIN/../lambdafs_amd'

# A/B of the staged pipeline's knobs, interleaved in one process (profiles/r06/).
tools/host_pipeline_sweep: tools/host_pipeline_sweep.cpp include/hrs.h $(LIB)
	g++ -O2 -std=c++17 -Wall -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include -o $@ $< -Llambdafs_amd -lhrs \
	    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN/../lambdafs_amd' -Wl,-rpath,/opt/rocm/lib

# Host copy rates of the staging copies on the box's CPUs (profiles/r06/).
tools/host_copy_probe: tools/host_copy_probe.cpp lambdafs_amd/csrc/hrs_host.hpp
	$(HIPCC) -O2 -std=c++17 -Wall -pthread -o $@ $<

$(API_OBJ): build/%.o: lambdafs_amd/csrc/%.cpp $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

build/hrs_kernels.o: lambdafs_amd/csrc/hrs_kernels.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_runtime.o: lambdafs_amd/csrc/hrs_runtime.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_batch.o: lambdafs_amd/csrc/hrs_batch.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_crc.o: lambdafs_amd/csrc/hrs_crc.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# The fused kernels' XOR networks and CRC steps must unroll completely (a
# K = 12 network otherwise stays a loop of runtime mask tests, 5x slower):
# lift the pragma-unroll size cap for this file.
build/hrs_fused.o: lambdafs_amd/csrc/hrs_fused.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -mllvm -pragma-unroll-threshold=1000000 -c $< -o $@

build/hrs_decode_crc.o: lambdafs_amd/csrc/hrs_decode_crc.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_gate.o: lambdafs_amd/csrc/hrs_gate.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_probe.o: lambdafs_amd/csrc/hrs_probe.hip include/hrs_probe.h $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

KOBJ     := build/hrs_kernels.o build/hrs_runtime.o build/hrs_batch.o build/hrs_crc.o build/hrs_fused.o build/hrs_decode_crc.o \
            build/hrs_gate.o

$(LIB): $(API_OBJ) $(KOBJ) lambdafs_amd/csrc/libhrs.map
	$(HIPCC) $(HIPFLAGS) -shared -Wl,--version-script=lambdafs_amd/csrc/libhrs.map -o $@ $(API_OBJ) $(KOBJ) \
	    -L/opt/rocm/lib -lhsa-runtime64

# HBM ceiling probes (include/hrs_probe.h): a side library for bench.py and
# tools only; the product libhrs.so does not carry diagnostics.
$(PROBE): build/hrs_probe.o lambdafs_amd/csrc/libhrs_probe.map
	$(HIPCC) $(HIPFLAGS) -shared -Wl,--version-script=lambdafs_amd/csrc/libhrs_probe.map -o $@ build/hrs_probe.o

$(ORACLE): oracle/rs_oracle.c oracle/rs_oracle.h
	$(CC) -O2 -std=c11 -fPIC -shared -Wall -Wextra -o $@ oracle/rs_oracle.c

# Test-only native harness (tests/cpp): the codec driven like Encoder/Decoder.
tests/cpp/codec_harness: tests/cpp/codec_harness.cpp include/hrs.hpp include/hrs.h $(LIB) $(ORACLE)
	g++ -O2 -std=c++17 -Wall -pthread -Iinclude -Ioracle -o $@ $< -Llambdafs_amd -lhrs -Loracle -loracle -lz \
	    -Wl,-rpath,'$$ORIGIN/../../lambdafs_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# The JNI shim, compiled against the hand-declared JNI ABI subset
# (lambdafs_amd/jni/jni_min.h; -DHRS_SYSTEM_JNI + JDK include dirs for <jni.h>).
$(JNI): lambdafs_amd/jni/hrs_jni.c lambdafs_amd/jni/jni_min.h include/hrs.h $(LIB)
	$(CC) -O2 -std=c11 -fPIC -shared -Wall -Wextra -Werror -Iinclude -o $@ $< -Llambdafs_amd -lhrs \
	    -Wl,-rpath,'$$ORIGIN'

# Fake-JVM harness driving every HrsNative entry point (tests/test_jni.py).
tests/cpp/jni_harness: tests/cpp/jni_harness.c lambdafs_amd/jni/jni_min.h $(JNI) $(ORACLE)
	$(CC) -O2 -std=c11 -Wall -Wextra -Iinclude -Ioracle -o $@ $< -Llambdafs_amd -lhrs_jni -lhrs -Loracle -loracle -lz -ldl \
	    -Wl,-rpath,'$$ORIGIN/../../lambdafs_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# Host-only logic (matrices, survivor lists, decode cache, batch plans) vs the oracle.
tests/cpp/host_logic: tests/cpp/host_logic.cpp include/hrs.h $(LIB) $(ORACLE)
	g++ -O2 -std=c++17 -Wall -Iinclude -Ioracle -o $@ $< -Llambdafs_amd -lhrs -Loracle -loracle \
	    -Wl,-rpath,'$$ORIGIN/../../lambdafs_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

# The CRC tables the kernels load, dumped for tests/test_crc_tables.py (host code;
# hipcc only for the HIP headers hrs_crc.hpp includes).
tests/cpp/crc_tables: tests/cpp/crc_tables.cpp lambdafs_amd/csrc/crc32.hpp lambdafs_amd/csrc/hrs_crc.hpp
	$(HIPCC) -O2 -std=c++17 -x hip --offload-arch=$(ARCH) -o $@ $<

# The host copy pool under concurrent callers (CPU only).
tests/cpp/copy_pool_test: tests/cpp/copy_pool_test.cpp lambdafs_amd/csrc/hrs_host.hpp
	g++ -O2 -std=c++17 -Wall -pthread -o $@ $<

tests/cpp/crc_model: tests/cpp/crc_model.cpp lambdafs_amd/csrc/crc32.hpp
	g++ -O2 -std=c++17 -Wall -o $@ $< -lz

# ---- make asan: the host-side code under AddressSanitizer + UBSan (clang,
# one runtime for all): libhrs's host logic (hrs_api.cpp, host code only: -Xarch_host),
# the oracle, the JNI shim, and the CPU drivers of each (host-only handles,
# the fake JVM). GPU kernels are not instrumented (no GPU ASan on this pool).
# Logs: profiles/r02/asan/.
ASAN_DIR := build/asan
CLANG    := /opt/rocm/lib/llvm/bin/clang
SAN      := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1
HSAN     := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
            -Xarch_host -fno-omit-frame-pointer
ASAN_BIN := $(ASAN_DIR)/host_logic $(ASAN_DIR)/jni_harness $(ASAN_DIR)/codec_harness
ASAN_LOG := profiles/r06/asan

ASAN_API := $(patsubst %,$(ASAN_DIR)/%.o,$(API_SRC))
$(ASAN_API): $(ASAN_DIR)/%.o: lambdafs_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) -O1 -g -std=c++17 -fPIC --offload-arch=$(ARCH) $(HSAN) -x hip -c $< -o $@

$(ASAN_DIR)/libhrs.so: $(ASAN_API) $(KOBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -fsanitize=address,undefined -o $@ $^

$(ASAN_DIR)/liboracle.so: oracle/rs_oracle.c oracle/rs_oracle.h
	@mkdir -p $(ASAN_DIR)
	$(CLANG) $(SAN) -std=c11 -fPIC -shared -o $@ oracle/rs_oracle.c

$(ASAN_DIR)/libhrs_jni.so: lambdafs_amd/jni/hrs_jni.c lambdafs_amd/jni/jni_min.h include/hrs.h $(ASAN_DIR)/libhrs.so
	$(CLANG) $(SAN) -std=c11 -fPIC -shared -Iinclude -o $@ $< -L$(ASAN_DIR) -lhrs

ASAN_RPATH := -Wl,-rpath,'$$ORIGIN'
$(ASAN_DIR)/host_logic: tests/cpp/host_logic.cpp $(ASAN_DIR)/libhrs.so $(ASAN_DIR)/liboracle.so
	$(CLANG)++ $(SAN) -std=c++17 -Iinclude -Ioracle -o $@ $< -L$(ASAN_DIR) -lhrs -loracle $(ASAN_RPATH)

$(ASAN_DIR)/jni_harness: tests/cpp/jni_harness.c $(ASAN_DIR)/libhrs_jni.so $(ASAN_DIR)/liboracle.so
	$(CLANG) $(SAN) -std=c11 -Iinclude -Ioracle -o $@ $< -L$(ASAN_DIR) -lhrs_jni -lhrs -loracle -lz -ldl $(ASAN_RPATH)

$(ASAN_DIR)/codec_harness: tests/cpp/codec_harness.cpp include/hrs.hpp $(ASAN_DIR)/libhrs.so $(ASAN_DIR)/liboracle.so
	$(CLANG)++ $(SAN) -std=c++17 -pthread -Iinclude -Ioracle -o $@ $< -L$(ASAN_DIR) -lhrs -loracle -lz $(ASAN_RPATH)

asan: $(ASAN_BIN)
	@mkdir -p $(ASAN_LOG)
	ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 LSAN_OPTIONS=suppressions=tools/lsan.supp \
	UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 sh -c '\
	  set -e; \
	  $(ASAN_DIR)/host_logic; \
	  $(ASAN_DIR)/jni_harness --cpu; \
	  for kp in "10 4" "12 4" "6 3" "3 2"; do $(ASAN_DIR)/codec_harness --host-only $$kp; done' \
	  > $(ASAN_LOG)/asan_run.log 2>&1 || { cat $(ASAN_LOG)/asan_run.log; exit 1; }
	@cat $(ASAN_LOG)/asan_run.log

# ---- make tsan: the host copy pool (hrs_host.hpp: concurrent callers,
# spinning workers that drain the batches they join) under ThreadSanitizer.
TSAN_LOG := profiles/r06/tsan
tsan: tests/cpp/copy_pool_test.cpp lambdafs_amd/csrc/hrs_host.hpp
	@mkdir -p build/tsan $(TSAN_LOG)
	g++ -O1 -g -std=c++17 -fsanitize=thread -pthread -o build/tsan/copy_pool_test tests/cpp/copy_pool_test.cpp
	sh -c 'for t in 0 1 4 8; do HRS_HOST_THREADS=$$t build/tsan/copy_pool_test 4 20; done' > $(TSAN_LOG)/tsan_run.log 2>&1 || { cat $(TSAN_LOG)/tsan_run.log; exit 1; }
	@cat $(TSAN_LOG)/tsan_run.log

clean:
	rm -rf build $(LIB) $(ORACLE) $(JNI) $(HARNESS) $(TOOLS)

.PHONY: all tsan clean asan
