# tests/native/asan.mk -- AddressSanitizer + UBSan builds of the product's HOST code (TEST
# INFRASTRUCTURE ONLY; SURVEY.md §4 item 5, mirroring the reference's Debug ASan build,
# CMakeLists.txt:47-48).  Outputs under tests/native/_build/asan/ (git-ignored):
#   dropin_cpu_asan   tests/native/dropin_cpu.cpp over the drop-in classes (resizers.cpp) with their
#                     CPU backend (cpu_generic.cpp) and the host plan (plan.cpp); the device side
#                     of the C ABI is tests/native/asan_nodevice.cpp (no gfx950 device)
#   host_tables_asan  tests/native/host_tables.cpp: every plan.cpp table builder, band windows and
#                     the kernels' table reads emulated (ratio_emul.cpp, tile_emul.cpp)
#   make -f tests/native/asan.mk [-j8]
ROOT  := $(abspath $(dir $(lastword $(MAKEFILE_LIST)))/../..)
OUT   ?= $(ROOT)/tests/native/_build/asan
CSRC  := $(ROOT)/libiqo_amd/csrc
CXX   ?= g++
SAN   := -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer
FLAGS := -std=c++17 -O1 -g $(SAN) -I$(ROOT)/include -I$(CSRC) -I/opt/rocm/include -D__HIP_PLATFORM_AMD__
# plan.cpp as the product builds it: strict IEEE (no contraction, no fast math)
STRICT := -ffp-contract=off -fno-fast-math

.PHONY: all
all: $(OUT)/dropin_cpu_asan $(OUT)/host_tables_asan

$(OUT)/%.o: $(CSRC)/%.cpp $(wildcard $(CSRC)/*.hpp) $(ROOT)/include/iqo_hip.h
	@mkdir -p $(OUT)
	$(CXX) $(FLAGS) $(STRICT) -c $< -o $@

$(OUT)/%.o: $(ROOT)/tests/native/%.cpp $(wildcard $(CSRC)/*.hpp) $(ROOT)/include/iqo_hip.h
	@mkdir -p $(OUT)
	$(CXX) $(FLAGS) $(STRICT) -c $< -o $@

$(OUT)/dropin_cpu_asan: $(OUT)/dropin_cpu.o $(OUT)/resizers.o $(OUT)/cpu_generic.o $(OUT)/plan.o $(OUT)/asan_nodevice.o
	$(CXX) $(SAN) -o $@ $^

$(OUT)/host_tables_asan: $(OUT)/host_tables.o $(OUT)/ratio_emul.o $(OUT)/tile_emul.o $(OUT)/plan.o
	$(CXX) $(SAN) -o $@ $^
