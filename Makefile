# Build for MI355X (gfx950).  `make` builds the engine and the oracle (test infrastructure).
# The packed-Shamir kernels are compiled as one object per instantiation family
# (SDA_GEN_PART / SDA_GEN_L = n+1 / k+t+1, SDA_REVEAL_PART = padded point count) so `make -j` builds them in parallel.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
EXTRA    ?=

CSRC    := sda_amd/csrc
OBJDIR  ?= build/obj
LIB     ?= sda_amd/libsda_engine.so

# share-gen objects, one per (n+1, k+t+1): the n+1 = 81 instantiations dominate the build, so they compile in parallel
GEN_PARTS    := 3_2 9_2 9_4 9_8 27_2 27_4 27_8 27_16 81_2 81_4 81_8 81_16 81_32 81_64
REVEAL_PARTS := 8 16 32 64 96
PLAIN   := combine elementwise chacha codec snapshot packed_wide
OBJS    := $(patsubst %,$(OBJDIR)/%.o,$(PLAIN)) $(OBJDIR)/engine.o \
           $(OBJDIR)/packed_gen.o $(patsubst %,$(OBJDIR)/packed_gen_%.o,$(GEN_PARTS)) \
           $(OBJDIR)/packed_reveal.o $(patsubst %,$(OBJDIR)/packed_reveal_%.o,$(REVEAL_PARTS))
HDRS    := $(CSRC)/packed_common.h $(CSRC)/kernels.h $(CSRC)/modarith.h $(CSRC)/xcd.h include/sda_engine.h

all: $(LIB) oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -c $< -o $@

$(OBJDIR)/packed_gen_%.o: $(CSRC)/packed_gen.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -DSDA_GEN_PART=$(word 1,$(subst _, ,$*)) -DSDA_GEN_L=$(word 2,$(subst _, ,$*)) -c $< -o $@

$(OBJDIR)/packed_reveal_%.o: $(CSRC)/packed_reveal.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -DSDA_REVEAL_PART=$* -c $< -o $@

$(OBJDIR)/engine.o: $(CSRC)/engine.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
