# Builds the in-tree HIP library for gfx950 (MI355X).  No cmake needed.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := super-resolution-climate_amd
SRC := $(PKG)/csrc
OUT := $(PKG)/srmi/libsrmi.so
OBJDIR := build/obj
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude
HIPSRC := $(SRC)/conv3x3.hip $(SRC)/wgrad3x3.hip $(SRC)/small.hip
CPPSRC := $(SRC)/engine.cpp
OBJS := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIPSRC)) $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.o,$(CPPSRC))
HDRS := $(SRC)/common.hpp $(SRC)/srmi_internal.hpp include/srmi.h

all: $(OUT)

$(OBJDIR)/%.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(OUT): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) $(OBJS) -o $@

oracle:
	@true

clean:
	rm -rf build $(OUT)

.PHONY: all clean oracle
