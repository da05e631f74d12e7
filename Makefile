# Builds the gfx950 engine (lambdafs_amd/libhrs.so) and the test-only CPU
# oracle (oracle/liboracle.so). `python -c "import __graft_entry__ as g; g.build()"`
# runs the same recipe.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CC       ?= gcc

LIB      := lambdafs_amd/libhrs.so
ORACLE   := oracle/liboracle.so
HDRS     := include/hrs.h lambdafs_amd/csrc/hrs_device.hpp lambdafs_amd/csrc/gf256.hpp lambdafs_amd/csrc/hrs_internal.hpp \
            lambdafs_amd/csrc/crc32.hpp lambdafs_amd/csrc/hrs_crc.hpp

JNI      := lambdafs_amd/libhrs_jni.so
HARNESS  := tests/cpp/codec_harness tests/cpp/crc_model tests/cpp/jni_harness

all: $(LIB) $(ORACLE) $(JNI) $(HARNESS)

build/hrs_api.o: lambdafs_amd/csrc/hrs_api.cpp $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

build/hrs_kernels.o: lambdafs_amd/csrc/hrs_kernels.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_crc.o: lambdafs_amd/csrc/hrs_crc.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

build/hrs_fused.o: lambdafs_amd/csrc/hrs_fused.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): build/hrs_api.o build/hrs_kernels.o build/hrs_crc.o build/hrs_fused.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

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
	$(CC) -O2 -std=c11 -Wall -Wextra -Iinclude -Ioracle -o $@ $< -Llambdafs_amd -lhrs_jni -lhrs -Loracle -loracle -lz \
	    -Wl,-rpath,'$$ORIGIN/../../lambdafs_amd' -Wl,-rpath,'$$ORIGIN/../../oracle'

tests/cpp/crc_model: tests/cpp/crc_model.cpp lambdafs_amd/csrc/crc32.hpp
	g++ -O2 -std=c++17 -Wall -o $@ $< -lz

clean:
	rm -rf build $(LIB) $(ORACLE) $(JNI) $(HARNESS)

.PHONY: all clean
