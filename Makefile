# Builds the product library (HIP, gfx950) and the CPU oracle (test infrastructure).
#   make            -> kmer-ml_amd/kmerml/_lib/libkmerhip.so + oracle/build/liboracle.so
#   make lib        -> product library only
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CSRC     := kmer-ml_amd/csrc
OUTDIR   := kmer-ml_amd/kmerml/_lib
OBJDIR   := $(CSRC)/build
LIB      := $(OUTDIR)/libkmerhip.so
OBJS     := $(OBJDIR)/kmh_api.o $(OBJDIR)/kmh_fasta.o $(OBJDIR)/kmh_dense.o $(OBJDIR)/kmh_sparse.o $(OBJDIR)/kmh_matrix.o $(OBJDIR)/kmh_hash.o $(OBJDIR)/kmh_io.o $(OBJDIR)/kmh_csv.o $(OBJDIR)/kmh_sort.o $(OBJDIR)/kmh_features.o $(OBJDIR)/kmh_shard.o $(OBJDIR)/kmh_wire.o
HDRS     := $(CSRC)/kmh_internal.h $(CSRC)/kmh_device.h include/kmerhip.h
SRCS     := $(wildcard $(CSRC)/*.hip $(CSRC)/*.cpp) $(HDRS)
# Build id: hash of every product source, compiled into kmh_build_id(); bench.py prints a
# PMC traffic figure only when profiles/pmc_traffic.json was measured on the same build id.
BUILD_ID := $(shell cat $(SRCS) | sha256sum | cut -c1-16)

all: lib oracle selftest

lib: $(LIB)

$(LIB): $(OBJS)
	@mkdir -p $(OUTDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS) -lz -lpthread

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(OBJDIR)/kmh_api.o: $(CSRC)/kmh_api.cpp $(SRCS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DKMH_BUILD_ID='"$(BUILD_ID)"' -x hip -c -o $@ $<

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(OBJDIR) $(OUTDIR)/libkmerhip.so
	$(MAKE) -C oracle clean

.PHONY: all lib oracle clean

SELFTEST := $(OUTDIR)/kmh_selftest
selftest: $(SELFTEST)

$(SELFTEST): tests/native/kmh_selftest.cpp $(LIB) include/kmerhip.h
	$(HIPCC) -O2 -std=c++17 -o $@ $< -L$(OUTDIR) -lkmerhip -Wl,-rpath,'$$ORIGIN'

.PHONY: selftest

LDSBENCH := $(OUTDIR)/lds_bench
ldsbench: $(LDSBENCH)
$(LDSBENCH): tests/native/lds_bench.hip
	@mkdir -p $(OUTDIR)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<
.PHONY: ldsbench

MALLBENCH := $(OUTDIR)/mall_bench
mallbench: $(MALLBENCH)
$(MALLBENCH): tests/native/mall_bench.hip
	@mkdir -p $(OUTDIR)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<
.PHONY: mallbench

FABBENCH := $(OUTDIR)/fabric_bench
fabbench: $(FABBENCH)
$(FABBENCH): tests/native/fabric_bench.hip
	@mkdir -p $(OUTDIR)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<
.PHONY: fabbench

RINGBENCH := $(OUTDIR)/ring_bench
ringbench: $(RINGBENCH)
$(RINGBENCH): tests/native/ring_bench.hip
	@mkdir -p $(OUTDIR)
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<
.PHONY: ringbench
