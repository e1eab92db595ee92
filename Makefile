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

all: $(LIB) $(CLI) oracle

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
VARIANTS := best pre0 prof pre0_prof
VFLAGS_pre0          := -DRTX_PREFILTER=0
VFLAGS_pre0_prof     := -DRTX_PREFILTER=0 -DRTX_DIAG_PROF=1
VFLAGS_best          := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=8
VFLAGS_blk64         := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=0 -DRTX_BLOCK=64
VFLAGS_blk128        := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_BLOCK=128
VFLAGS_blk64_w7      := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_BLOCK=64 -DRTX_WAVES_PER_SIMD=7
VFLAGS_lpt           := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1
VFLAGS_lpt_blk64     := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_BLOCK=64
VFLAGS_lpt_r0        := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_RADIUS=0
VFLAGS_lpt_r2        := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_RADIUS=2
VFLAGS_lpt_s2        := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_SPP=2
VFLAGS_lpt_cw4       := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_CW=4
VFLAGS_lpt_s2_cw4    := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_SPP=2 -DRTX_LPT_CW=4
VFLAGS_lpt_b1k       := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_BUCKETS=1024
VFLAGS_lpt_b1k_r2    := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_BUCKETS=1024 -DRTX_LPT_RADIUS=2
VFLAGS_lpt_b1k_cw4   := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_BUCKETS=1024 -DRTX_LPT_CW=4
VFLAGS_lpt_b1k_s2    := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_LPT_BUCKETS=1024 -DRTX_LPT_SPP=2
VFLAGS_lpt_coop4     := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=4
VFLAGS_lpt_coop8     := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=8
VFLAGS_lpt_coop16    := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=16
VFLAGS_blk64_coop8   := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=0 -DRTX_BLOCK=64 -DRTX_COOP_MAX=8
VFLAGS_merge         := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=8 -DRTX_SHADE_MERGE=1
VFLAGS_prof          := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=8 -DRTX_DIAG_PROF=1
VFLAGS_prof_merge    := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_COOP_MAX=8 -DRTX_DIAG_PROF=1 -DRTX_SHADE_MERGE=1
VFLAGS_lpt_blk128    := -DRTX_DEFER=1 -DRTX_SRC=1 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1 -DRTX_PERSISTENT=1 -DRTX_BLOCK=128
VFLAGS_lds_stream_b8 := -DRTX_DEFER=1 -DRTX_SRC=0 -DRTX_BATCH=8 -DRTX_LISTMASK=1 -DRTX_ANYMAX=1
VDIR := $(LIBDIR)/variants

variants: $(foreach v,$(VARIANTS),$(VDIR)/librtx_$(v).so)

$(VDIR)/librtx_%.so: $(SRC)/rtx_kernels.hip $(SRC)/rtx_api.hip $(SRC)/rtx_host.cpp $(HDRS)
	mkdir -p $(VDIR)/$*
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_kernels.hip -o $(VDIR)/$*/k.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_api.hip -o $(VDIR)/$*/a.o
	$(HIPCC) $(HIPFLAGS) $(VFLAGS_$*) -c $(SRC)/rtx_host.cpp -o $(VDIR)/$*/h.o
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(VDIR)/$*/k.o $(VDIR)/$*/a.o $(VDIR)/$*/h.o

.PHONY: variants
