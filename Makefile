# zkmi developer entry points (the role of the reference's Makefile /
# tools/mk: all, test, check).  GPU targets need an MI355X (run them through
# gpurun on this pool).
PY ?= python

.PHONY: all build test test-gpu check lint sanitize bench bench-all prof clean

all: build

build:                    ## HIP kernels (gfx950) + C++ host codec, in-tree
	$(PY) tools/build_native.py

test:                     ## CPU suite (fake ZooKeeper, gloo, host codec)
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu:                 ## kernel numerics + GPU pipelines (needs a GPU)
	$(PY) -m pytest tests -x -q -m gpu

check: lint sanitize      ## style + sanitizer runs

lint:
	$(PY) tools/lint.py

sanitize:                 ## host codec suites under ASan + UBSan
	bash tools/sanitize_host.sh

bench:                    ## headline benchmark, 1 GPU
	$(PY) bench.py

bench-all:                ## gpu tests + get / mix / storm workloads (needs a GPU)
	bash tools/gpu.sh tests bench=--no-rtt bench=--no-rtt,--workload,mix \
	  bench=--no-rtt,--workload,storm

prof:                     ## rocprofv3 kernel stats for the three workloads
	bash tools/gpu.sh prof=prof,get,mix,storm

clean:
	rm -rf build zkmi/ops/libzkmi_hip.so zkmi/_zkhost*.so
