"""Interpreter start-up hook that enforces a GPU share's HBM cap.

``python -m kgwe.launch`` puts this directory first on PYTHONPATH when the
placement carries ``KGWE_GPU_MEMORY_FRACTION``.  Nothing is imported here
beyond the standard library: the hook waits for the workload's own ``import
torch`` and then queues ``set_per_process_memory_fraction`` for every visible
device on torch's lazy CUDA/HIP initialisation, so the cap is in place before
the process can allocate — whether or not the workload knows about kgwe
(reference MPS memory limit: recorded, enforced nowhere,
src/sharing/mig_controller.go:594-678).  An allocation past the cap raises
``torch.OutOfMemoryError`` in that client; its neighbours on the GPU are not
touched.
"""
import os
import sys


def _chain():
    """Run the sitecustomize this one shadows, if there is one."""
    here = os.path.dirname(os.path.abspath(__file__))
    for p in sys.path:
        if not p or os.path.abspath(p) == here:
            continue
        f = os.path.join(p, "sitecustomize.py")
        if os.path.isfile(f):
            import importlib.util

            spec = importlib.util.spec_from_file_location("_kgwe_chained_sitecustomize", f)
            if spec and spec.loader:
                spec.loader.exec_module(importlib.util.module_from_spec(spec))
            return


def _cap(torch, frac):
    def apply():
        for d in range(torch.cuda.device_count()):
            torch.cuda.set_per_process_memory_fraction(frac, d)

    try:
        torch.cuda._lazy_call(apply)  # runs inside torch's lazy init (or now, if it already ran)
        os.environ["KGWE_GPU_MEMORY_CAP_INSTALLED"] = "1"
    except Exception as e:  # noqa: BLE001 - a torch without this hook: say so, do not break the workload
        print(f"[kgwe] could not install the HBM cap: {e}", file=sys.stderr)


def _install():
    try:
        frac = float(os.environ.get("KGWE_GPU_MEMORY_FRACTION", "0") or 0)
    except ValueError:
        return
    if not 0.0 < frac < 1.0:
        return
    import importlib.abc
    import importlib.util

    class _TorchHook(importlib.abc.MetaPathFinder):
        def find_spec(self, name, path, target=None):
            if name != "torch":
                return None
            sys.meta_path.remove(self)
            spec = importlib.util.find_spec("torch")
            if spec is None or spec.loader is None:
                return spec
            run = spec.loader.exec_module

            def exec_module(module):
                run(module)
                _cap(module, frac)

            spec.loader.exec_module = exec_module
            return spec

    sys.meta_path.insert(0, _TorchHook())


_install()
try:
    _chain()
except Exception as e:  # noqa: BLE001
    print(f"[kgwe] chained sitecustomize failed: {e}", file=sys.stderr)
