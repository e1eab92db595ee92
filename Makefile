# Build for the MI355X-native path tracer (gfx950) and its CPU oracle.
#   make            -> librtx.so + rtx_cli + liboracle.so (+ oracle/_ref when /root/reference exists)
# -ffp-contract=off everywhere: fused multiply-adds only where written as fmaf,
# so the HIP kernel and the C oracle execute the same IEEE op sequence.
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
PKG       := raytrace-we-gpu_amd
SRC       := $(PKG)/csrc
LIBDIR    := $(PKG)/lib
BINDIR    := $(PKG)/bin
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden -ffp-contract=off -Wall -Wno-unused-function
LIB       := $(LIBDIR)/librtx.so
CLI       := $(BINDIR)/rtx_cli
HDRS      := include/rtx.h $(SRC)/rtx_internal.h $(SRC)/rtx_device_math.h $(SRC)/rtx_prefilter.h $(SRC)/rtx_grid.h
# Build provenance (rtx_build_info): the library records the hash of the
# sources it was built from; bench.py compares it with the tree's
# (tools/src_sha.py computes the same hash).
LIBSRCS   := $(sort $(wildcard $(SRC)/*.hip $(SRC)/*.h $(SRC)/*.cpp)) include/rtx.h
SRC_SHA   := $(shell python3 tools/src_sha.py)

UBENCH    := tools/ubench_issue

all: $(LIB) $(CLI) oracle $(LIBDIR)/variants/librtx_stress.so $(UBENCH)

# VALU issue cost per instruction class in the chip's own cycles (bench.py's
# issue ceiling, tools/issue_probe.py)
$(UBENCH): tools/ubench_issue.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<

$(LIBDIR)/%.o: $(SRC)/%.hip $(HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# rtx_api.o carries the source hash: rebuilt whenever any library source changes
$(LIBDIR)/rtx_api.o: $(SRC)/rtx_api.hip $(LIBSRCS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DRTX_SRC_SHA='"$(SRC_SHA)"' -c $< -o $@

$(LIBDIR)/rtx_host.o: $(SRC)/rtx_host.cpp include/rtx.h | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(LIBDIR)/rtx_kernels.o $(LIBDIR)/rtx_api.o $(LIBDIR)/rtx_host.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

$(CLI): $(SRC)/rtx_cli.cpp $(SRC)/rtx_app.cpp include/rtx.h include/rtx_app.hpp $(LIB) | $(BINDIR)
	$(HIPCC) -O2 -std=c++17 -ffp-contract=off -Wall -o $@ $(SRC)/rtx_cli.cpp $(SRC)/rtx_app.cpp \
	    -L$(LIBDIR) -lrtx -Wl,-rpath,'$$ORIGIN/../lib' -lpthread

$(LIBDIR) $(BINDIR):
	mkdir -p $@

oracle:
	$(MAKE) -C oracle

asm: | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) --offload-device-only -S $(SRC)/rtx_kernels.hip -o $(LIBDIR)/rtx_kernels.s

clean:
	rm -rf $(LIBDIR) $(BINDIR)
	$(MAKE) -C oracle clean

.PHONY: all oracle asm clean

# Kernel variants (same sources, different compile-time choices; never the
# product path):
#   stress - candidate lists of 1 entry and coop resolve rounds of one scan
#            step, so every overflow, round and fallback path runs all the
#            time, and a 20 ms promotion valve (the heartbeat keeps live
#            launches going), and the kernarg layout check (RTX_CHECK_KERNARG)
#            (tests/test_gpu_parity.py)
#   prof   - per-section clock sums (tools/section_prof.py)
#   ptime  - per-pixel start/end times (tools/pixel_timeline.py)
#   cprof  - per-section clocks of tier-1 coop segments (tools/coop_prof.py)
#   rays   - a sample of lane-mode wave iterations' rays (tools/ray_sample.py)
# Ad-hoc A/B builds for tools/variant_bench.py:
#   make adhoc V=name VFLAGS="-DRTX_...=..."   -> lib/variants/librtx_name.so
VARIANTS := stress prof ptime cprof rays
VFLAGS_stress        := -DRTX_CAND=1 -DRTX_CAND_PF=1 -DRTX_GF_STEPS=1 -DRTX_PROM_VALVE_TICKS=2000000ull -DRTX_CHECK_KERNARG=1
VFLAGS_prof          := -DRTX_DIAG_PROF=1
VFLAGS_ptime         := -DRTX_DIAG_PIXEL=1
VFLAGS_cprof         := -DRTX_DIAG_COOP=1
VFLAGS_rays          := -DRTX_DIAG_RAYS=4099
VDIR := $(LIBDIR)/variants

variants: $(foreach v,$(VARIANTS),$(VDIR)/librtx_$(v).so)

$(VDIR)/librtx_%.so: $(SRC)/rtx_kernels.hip $(SRC)/rtx_api.hip $(SRC)/rtx_host.cpp $(HDRS) Makefile
	mkdir -p $(VDIR)/$*
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_kernels.hip -o $(VDIR)/$*/k.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -DRTX_SRC_SHA='"$(SRC_SHA)"' -DRTX_VARIANT='"$*"' -c $(SRC)/rtx_api.hip -o $(VDIR)/$*/a.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_host.cpp -o $(VDIR)/$*/h.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(VDIR)/$*/k.o $(VDIR)/$*/a.o $(VDIR)/$*/h.o

adhoc:
	@test -n "$(V)" || (echo "usage: make adhoc V=name VFLAGS=..." && false)
	mkdir -p $(VDIR)/$(V)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $(SRC)/rtx_kernels.hip -o $(VDIR)/$(V)/k.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -DRTX_VARIANT='"$(V)"' -c $(SRC)/rtx_api.hip -o $(VDIR)/$(V)/a.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $(SRC)/rtx_host.cpp -o $(VDIR)/$(V)/h.o
	$(HIPCC) $(HIPFLAGS) -shared -o $(VDIR)/librtx_$(V).so $(VDIR)/$(V)/k.o $(VDIR)/$(V)/a.o $(VDIR)/$(V)/h.o

.PHONY: variants adhoc
