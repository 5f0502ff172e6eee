# Top-level build: the HIP E-step library (gfx950), the oracle (C restatement,
# test infrastructure), and the test-only MATLAB API double + MEX gateway.
PKG      := clustering-hidden-markov-models-with-variational-bayesian-hierarchical-em_amd
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-function
LIBDIR   := $(PKG)/lib
SRCS     := $(PKG)/csrc/vbhem_kernels.hip $(PKG)/csrc/vbhem_fb_split.hip $(PKG)/csrc/vbhem_fb_bwd.hip $(PKG)/csrc/vbhem_fb_bwd4.hip $(PKG)/csrc/vbhem_fb_bwd12.hip $(PKG)/csrc/vbhem_fb_list4.hip $(PKG)/csrc/vbhem_fb_list12.hip $(PKG)/csrc/vbhem_emission.hip $(PKG)/csrc/vbhem_stats.hip $(PKG)/csrc/vbhem_capi.hip $(PKG)/csrc/vbhem_em.hip $(PKG)/csrc/vbhem_em_dev.hip $(PKG)/csrc/vbhem_rccl.hip $(PKG)/csrc/vbhem_h3m.hip $(PKG)/csrc/vbhmm_fb.hip
HDRS     := include/vbhem_estep.h include/vbhem_dist.h include/vbhmm_fb.h $(PKG)/csrc/vbhem_internal.h $(PKG)/csrc/vbhem_math.h $(PKG)/csrc/vbhem_log_table.h include/vbhem_em.h $(PKG)/csrc/vbhem_em_dev.h $(PKG)/csrc/vbhem_exact.h $(PKG)/csrc/vbhem_mfma4.h
OBJS     := $(patsubst $(PKG)/csrc/%.hip,$(LIBDIR)/%.o,$(SRCS))

all: lib oracle mex mathcheck

lib: $(LIBDIR)/libvbhem_estep.so

$(LIBDIR)/%.o: $(PKG)/csrc/%.hip $(HDRS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -Iinclude -I$(PKG)/csrc -c -o $@ $<

$(LIBDIR)/libvbhem_estep.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle liboracle.so

# test-only: a MATLAB mx/mex API double and the MEX gateway built against it
mex: tests/mxshim/libmxshim.so $(LIBDIR)/vbhem_hmm_bwd_fwd_mex.so $(LIBDIR)/hem_hmm_bwd_fwd_mex.so $(LIBDIR)/vbhmm_fb_mex.so $(LIBDIR)/vbhem_estep_fused_mex.so

tests/mxshim/libmxshim.so: tests/mxshim/mxshim.c tests/mxshim/mex.h
	gcc -O2 -fPIC -shared -Itests/mxshim -o $@ $<

$(LIBDIR)/%_mex.so: integration/%_mex.c integration/h3m_mex_common.h include/vbhem_estep.h include/vbhmm_fb.h $(LIBDIR)/libvbhem_estep.so tests/mxshim/mex.h
	gcc -O2 -fPIC -shared -Iinclude -Itests/mxshim -Iintegration -o $@ $< -L$(LIBDIR) -lvbhem_estep -lm -Wl,-rpath,'$$ORIGIN'

# test-only: the restricted-domain exp/log/rcp of vbhem_math.h, host and device
mathcheck: tests/mathcheck/libmathcheck.so

tests/mathcheck/libmathcheck.so: tests/mathcheck/mathcheck.hip $(PKG)/csrc/vbhem_math.h $(PKG)/csrc/vbhem_log_table.h $(PKG)/csrc/vbhem_mfma4.h
	$(HIPCC) $(HIPFLAGS) -I$(PKG)/csrc -shared -o $@ $<

clean:
	rm -f $(LIBDIR)/*.o $(LIBDIR)/*.so tests/mxshim/libmxshim.so tests/mathcheck/libmathcheck.so
	$(MAKE) -C oracle clean

.PHONY: all lib oracle mex mathcheck clean
