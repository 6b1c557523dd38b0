# tests/native/dropin.mk -- source-level drop-in proof (TEST INFRASTRUCTURE ONLY).
#
# Compiles the reference's own tools UNCHANGED, from where they lie under $(REF), against this
# repo's public headers (include/libiqo) and libiqo_amd/libiqo_hip.so instead of the reference's
# libiqo.a:
#   $(REF)/benchmark/benchmark.cpp      (its CMake flags: -std=c++11 -Ofast, benchmark/CMakeLists.txt:23-40)
#   $(REF)/sample/resize_yuv420p.cpp    (-std=c++98 -fno-exceptions, sample/CMakeLists.txt:5-6)
# config.h is generated from benchmark/config.h.in the way CMake's configure_file does when
# neither OpenCV nor IPP is found (benchmark/CMakeLists.txt:64-92): every #cmakedefine becomes
# an #undef.  Nothing of the reference is copied; outputs go to $(OUT) only (git-ignored).
#   make -f tests/native/dropin.mk [REF=/root/reference] [OUT=tests/native/_build/dropin]
REF  ?= /root/reference
ROOT := $(abspath $(dir $(lastword $(MAKEFILE_LIST)))/../..)
OUT  ?= $(ROOT)/tests/native/_build/dropin
CXX  ?= g++
LIB  := $(ROOT)/libiqo_amd
LINK := -L$(LIB) -liqo_hip -Wl,-rpath,'$$ORIGIN/../../../../libiqo_amd' -Wl,-rpath,/opt/rocm/lib \
        -Wl,-rpath-link,/opt/rocm/lib

.PHONY: all
all: $(OUT)/benchmark $(OUT)/resize_yuv420p

$(OUT)/config.h: $(REF)/benchmark/config.h.in
	mkdir -p $(OUT)
	sed -e 's|^#cmakedefine[ ]*\([A-Za-z0-9_]*\).*$$|/* #undef \1 */|' $< > $@

$(OUT)/benchmark: $(REF)/benchmark/benchmark.cpp $(OUT)/config.h $(LIB)/libiqo_hip.so $(wildcard $(ROOT)/include/libiqo/*.hpp)
	$(CXX) -std=c++11 -O3 -Ofast -w -I$(ROOT)/include -I$(OUT) -o $@ $< $(LINK)

$(OUT)/resize_yuv420p: $(REF)/sample/resize_yuv420p.cpp $(LIB)/libiqo_hip.so $(wildcard $(ROOT)/include/libiqo/*.hpp)
	mkdir -p $(OUT)
	$(CXX) -std=c++98 -fno-exceptions -O3 -w -I$(ROOT)/include -o $@ $< $(LINK)
