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
HDRS      := include/rtx.h $(SRC)/rtx_internal.h $(SRC)/rtx_device_math.h $(SRC)/rtx_prefilter.h

all: $(LIB) $(CLI) oracle $(LIBDIR)/variants/librtx_stress.so

$(LIBDIR)/%.o: $(SRC)/%.hip $(HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

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

# Kernel variants for A/B timing (tools/variant_bench.py): same sources,
# different compile-time choices. Not used by the product path.
VARIANTS := best nopack w4 w6 lag0 lag32 every4 noflat prof ptime cprof cprof2 stress cand24 cand6 pfcand12 ps1024 ps256 ps128 psb80 psb20
VFLAGS_best          :=
VFLAGS_noflat        := -DRTX_FLAT=0
VFLAGS_nopack        := -DRTX_PACK=0
VFLAGS_w4            := -DRTX_WAVES_PER_SIMD=4
VFLAGS_w6            := -DRTX_WAVES_PER_SIMD=6
VFLAGS_lag0          := -DRTX_PACK_LAG=0
VFLAGS_lag32         := -DRTX_PACK_LAG=32
VFLAGS_every4        := -DRTX_PACK_EVERY=4
VFLAGS_prof          := -DRTX_DIAG_PROF=1
VFLAGS_ptime         := -DRTX_DIAG_PIXEL=1
VFLAGS_cprof         := -DRTX_DIAG_COOP=1
VFLAGS_cprof2        := -DRTX_DIAG_COOP=2
# candidate-list length (entries of 8 spheres per lane before a resolve round)
VFLAGS_cand24        := -DRTX_CAND=24
VFLAGS_cand6         := -DRTX_CAND=6
VFLAGS_pfcand12      := -DRTX_CAND_PF=12
# per-sample kernel: items per batch slot, batches per wave
VFLAGS_ps1024        := -DRTX_PS_ITEMS=1024
VFLAGS_ps256         := -DRTX_PS_ITEMS=256
VFLAGS_ps128         := -DRTX_PS_ITEMS=128
VFLAGS_psb80         := -DRTX_PS_BPW=80
VFLAGS_psb20         := -DRTX_PS_BPW=20
# test build: lists of 1 entry and 2 sphere-major pairs, so every overflow and
# fallback path runs all the time (tests/test_gpu_parity.py, stress tests)
VFLAGS_stress        := -DRTX_CAND=1 -DRTX_CAND_PF=1 -DRTX_SM_CAND=2
VDIR := $(LIBDIR)/variants

variants: $(foreach v,$(VARIANTS),$(VDIR)/librtx_$(v).so)

$(VDIR)/librtx_%.so: $(SRC)/rtx_kernels.hip $(SRC)/rtx_api.hip $(SRC)/rtx_host.cpp $(HDRS)
	mkdir -p $(VDIR)/$*
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_kernels.hip -o $(VDIR)/$*/k.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_api.hip -o $(VDIR)/$*/a.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_host.cpp -o $(VDIR)/$*/h.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(VDIR)/$*/k.o $(VDIR)/$*/a.o $(VDIR)/$*/h.o

.PHONY: variants
