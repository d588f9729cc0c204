# Convenience targets (reference: allreduce_over_mpi/Makefile — `make build` + `make sync` scp to 16 hosts).
#   make build            libflexar.so (gfx950) + C++ tools (bin/)
#   make test             CPU test suite          make test-gpu   GPU suite (on an MI355X)
#   make bench N=8        torchrun bench.py over N local GPUs
#   make mpi-bench N=2    MPI driver (host buffers) — reference benchmark.cpp CLI
#   make sync HOSTS=hostfile   rsync the built tree to every host listed (host[:slots] per line)
PY ?= python
N ?= 8
HOSTS ?= hostfile
DEST ?= $(CURDIR)

.PHONY: build test test-gpu bench mpi-bench sync clean

build:
	$(PY) -c "from allreduce_over_mpi_amd import _build; _build.build(verbose=True); print(_build.build_tools())"

test: build
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu: build
	$(PY) -m pytest tests -q -m gpu

bench: build
	$(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $(N) --master-addr 127.0.0.1 --master-port 29511 \
		bench.py --gpus $(N)

mpi-bench: build
	/opt/conda/bin/mpirun -np $(N) bin/flexar_bench --mem host --size 1024 --repeat 200

sync: build
	@for h in $$(cut -d: -f1 $(HOSTS) | grep -v '^#'); do \
		echo "sync -> $$h:$(DEST)"; rsync -a --exclude .git --exclude build $(CURDIR)/ $$h:$(DEST)/ || exit 1; \
	done

clean:
	rm -rf build bin allreduce_over_mpi_amd/_lib
