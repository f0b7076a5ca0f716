# Builds the in-tree HIP library for gfx950 (MI355X).  No cmake needed.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := super-resolution-climate_amd
SRC := $(PKG)/csrc
OUT := $(PKG)/srmi/libsrmi.so
OBJDIR ?= build/obj
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude $(EXTRA)
HIPSRC := $(SRC)/conv3x3.hip $(SRC)/conv_f32.hip $(SRC)/wgrad3x3.hip $(SRC)/small.hip $(SRC)/tiles.hip $(SRC)/rcab_infer.hip
CPPSRC := $(SRC)/engine.cpp
OBJS := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIPSRC)) $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.o,$(CPPSRC))
HDRS := $(SRC)/tuning.hpp $(SRC)/common.hpp $(SRC)/srmi_internal.hpp $(SRC)/conv64_body.hpp $(SRC)/wgrad_reduce.hpp $(SRC)/ca_scale.hpp include/srmi.h

all: $(OUT)

$(OBJDIR)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(OUT): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJS) -o $@

# diagnostic build with s_memtime phase stamps (tools/kbench.py KBENCH_STAMPS=1)
STAMPOBJDIR := build/obj_stamps
STAMPOUT := $(PKG)/srmi/libsrmi_stamps.so
STAMPOBJS := $(patsubst $(SRC)/%.hip,$(STAMPOBJDIR)/%.o,$(HIPSRC)) $(patsubst $(SRC)/%.cpp,$(STAMPOBJDIR)/%.o,$(CPPSRC))

$(STAMPOBJDIR)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(STAMPOBJDIR)
	$(HIPCC) $(CXXFLAGS) -DSRMI_STAMPS -c $< -o $@

$(STAMPOBJDIR)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(STAMPOBJDIR)
	$(HIPCC) $(CXXFLAGS) -DSRMI_STAMPS -c $< -o $@

$(STAMPOUT): $(STAMPOBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(STAMPOBJS) -o $@

stamps: $(STAMPOUT)

oracle:
	@true

clean:
	rm -rf build $(OUT) $(STAMPOUT)

.PHONY: all clean oracle stamps
