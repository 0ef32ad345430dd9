# ASan + UBSan build of the host code that parses untrusted input: both OBJ/MTL loaders, the BVH
# builder and the oracle (CPU only; GPU sanitizers are not available on this pool). Output goes to
# $(OUT) (default: a build directory outside the source tree).
#   make -f tests/sanitize.mk OUT=/tmp/rt_san    ->  $(OUT)/loader_san
ROOT    := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))..
OUT     ?= $(ROOT)/raytracert_amd/build/san
SAN     := -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1
CXXFLAGS := -std=c++17 -ffp-contract=off -fno-fast-math -pthread $(SAN) -I$(ROOT)/include \
            -I$(ROOT)/raytracert_amd/csrc -I$(ROOT)/oracle
CFLAGS  := -std=gnu11 -ffp-contract=off -fno-fast-math -pthread $(SAN)
SRCS    := $(ROOT)/raytracert_amd/csrc/scene_loader.cpp $(ROOT)/raytracert_amd/csrc/obj_parallel.cpp \
           $(ROOT)/raytracert_amd/csrc/bvh.cpp $(ROOT)/tests/cxx/loader_san.cpp

$(OUT)/loader_san: $(SRCS) $(OUT)/rt_oracle.o
	g++ $(CXXFLAGS) -o $@ $(SRCS) $(OUT)/rt_oracle.o -lm

$(OUT)/rt_oracle.o: $(ROOT)/oracle/rt_oracle.c $(ROOT)/oracle/rt_oracle.h
	@mkdir -p $(OUT)
	gcc $(CFLAGS) -c -o $@ $<
