# Build for MI355X (gfx950).  `make` builds the engine and the oracle (test infrastructure).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
JOBS     ?= 8

CSRC    := sda_amd/csrc
OBJDIR  := build/obj
SRCS    := $(CSRC)/combine.hip $(CSRC)/elementwise.hip $(CSRC)/packed_gen.hip $(CSRC)/packed_reveal.hip $(CSRC)/chacha.hip
OBJS    := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRCS)) $(OBJDIR)/engine.o
HDRS    := $(CSRC)/packed_common.h $(CSRC)/kernels.h $(CSRC)/modarith.h include/sda_engine.h
LIB     := sda_amd/libsda_engine.so

all: $(LIB) oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/engine.o: $(CSRC)/engine.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

tests-cpp: $(LIB)
	$(MAKE) -C tests/cpp

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean tests-cpp
