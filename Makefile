# Developer targets (the reference's CONTRIBUTING.md promises `make lint`; its Makefile is empty).
PY ?= python

.PHONY: build test test-gpu lint smoke bench clean

build:           ## compile csrc/ for gfx950 into ddlb_amd/_C*.so (in-tree)
	$(PY) -m ddlb_amd._build

test:            ## CPU suite (gloo multi-process tests included)
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu:        ## GPU suite on an MI355X
	$(PY) -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread

lint:
	$(PY) scripts/lint.py

smoke:
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

bench:
	$(PY) bench.py

clean:
	rm -rf build/native ddlb_amd/_C*.so
