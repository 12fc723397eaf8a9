# kgwe-mi355x developer targets (reference: Makefile:1-224 — Go build/test/lint,
# controller-gen, docker, helm).  Everything native is built by kgwe/_build.py
# (hipcc --offload-arch=gfx950 for the kernels, g++ + pybind11 for the core).
PY      ?= python
IMAGE   ?= kgwe/kgwe-mi355x
TAG     ?= dev
NPROC   ?= 8

.PHONY: all build rebuild test test-gpu test-all bench bench-sched busbw crds dashboard \
        helm-lint docker clean sanitize native-tests

all: build test

build:                     ## compile HIP kernels, probes and the C++ core in-tree
	$(PY) -m kgwe build -j $(NPROC)

rebuild:
	$(PY) -m kgwe build --force -j $(NPROC)

test: build                ## CPU suite (scheduler, partitions, cost, e2e, DP over gloo)
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu: build            ## MI355X suite (kernel numerics vs fp32 references, probes)
	timeout -k 10 1200 $(PY) -m pytest tests -q -m gpu

test-all: test test-gpu

bench: build               ## headline JSON line on one GPU
	timeout -k 10 1200 $(PY) bench.py --steps 10 --warmup 3

bench-sched:               ## scheduling latency only (CPU)
	$(PY) -m kgwe bench-sched --json

busbw: build               ## RCCL all-reduce bus bandwidth sweep over local GPUs
	$(PY) -m kgwe busbw

crds:                      ## re-render CRD YAML from kgwe/api/crds.py
	$(PY) -m kgwe crds deploy/helm/kgwe-mi355x/crds

dashboard:                 ## re-render the Grafana dashboard JSON
	$(PY) deploy/monitoring/gen_dashboard.py

helm-lint: crds dashboard
	helm lint deploy/helm/kgwe-mi355x
	helm template kgwe deploy/helm/kgwe-mi355x > /dev/null

docker:
	docker build -f docker/Dockerfile -t $(IMAGE):$(TAG) .

native-tests:              ## standalone C++ core tests: plain, TSan, ASan+UBSan builds
	$(PY) -m kgwe._build --native-tests plain --native-tests tsan --native-tests asan -j $(NPROC)
	./build/tests/core_tests_plain 2000
	TSAN_OPTIONS=halt_on_error=1 ./build/tests/core_tests_tsan 400
	ASAN_OPTIONS=halt_on_error=1 ./build/tests/core_tests_asan 400

sanitize:                  ## host-side ASan/UBSan build of the C++ core + CPU tests
	KGWE_CORE_SANITIZE=1 $(PY) -m kgwe build --force -j $(NPROC)
	ASAN_OPTIONS=detect_leaks=0 LD_PRELOAD=$$(g++ -print-file-name=libasan.so) \
	  $(PY) -m pytest tests -q -m "not gpu" -p no:cacheprovider
	$(PY) -m kgwe build --force -j $(NPROC)

clean:
	rm -rf kgwe/_lib build
