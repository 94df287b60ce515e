# Build libskm (HIP, gfx950), the host CLIs, and the CPU oracle (test infrastructure).
#   make            -> signature_kmers_amd/libskm.so, bin/kmers-*, oracle/liboracle_skm.so
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
ARCH    ?= gfx950
JOBS    ?= 8
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -ffp-contract=off -DSKM_WITH_RCCL \
           -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Wall -Wno-unused-function
OBJDIR   = build/obj
SRC      = signature_kmers_amd/csrc
HIP_SRCS = $(SRC)/skm_build.hip $(SRC)/skm_annotate.hip $(SRC)/skm_matrix.hip $(SRC)/skm_output.hip
CPP_SRCS = $(SRC)/skm_host.cpp $(SRC)/skm_bdz.cpp
OBJS     = $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS)) $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.o,$(CPP_SRCS))
LIB      = signature_kmers_amd/libskm.so
TOOLS    = bin/kmers-build-signatures bin/kmers-call-functions bin/kmers-annotate-seqs bin/kmers-matrix-distance bin/skm-front-probe
ORACLE   = oracle/liboracle_skm.so
FRONT    = $(OBJDIR)/front/skm_front.o $(OBJDIR)/front/skm_caller.o $(OBJDIR)/front/skm_mesh.o
FRONTH   = $(wildcard $(SRC)/front/*.h) $(SRC)/skm_strutil.h include/skm.h

all: $(LIB) $(ORACLE) $(TOOLS)
tools: $(TOOLS)

$(OBJDIR)/%.o: $(SRC)/%.hip $(wildcard $(SRC)/*.h) include/skm.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.cpp $(wildcard $(SRC)/*.h) include/skm.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS) -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# host front end + CLIs: plain C++ over the C-ABI (no HIP in these translation units)
$(OBJDIR)/front/%.o: $(SRC)/front/%.cpp $(FRONTH)
	@mkdir -p $(OBJDIR)/front
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -I$(SRC)/front -c $< -o $@

bin/%: $(SRC)/tools/%.cpp $(FRONT) $(LIB) $(FRONTH)
	@mkdir -p bin
	$(CXX) -O2 -std=c++17 -Wall -Iinclude -I$(SRC)/front $< $(FRONT) -o $@ -L signature_kmers_amd -lskm -pthread \
	  -Wl,-rpath,'$$ORIGIN/../signature_kmers_amd' -Wl,-rpath,/opt/rocm/lib

# random-gather ceiling of the annotate lookup (not part of `all`)
probe: bin/gather_probe
bin/gather_probe: tools/gather_probe.cpp
	@mkdir -p bin
	$(HIPCC) --offload-arch=$(ARCH) -O3 -x hip $< -o $@

$(ORACLE): oracle/skm_oracle.cpp
	$(CXX) -O2 -fPIC -shared -std=c++17 -ffp-contract=off -pthread $< -o $@

clean:
	rm -rf build bin $(LIB) $(ORACLE)

.PHONY: all clean probe
