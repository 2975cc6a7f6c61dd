"""Migrate the reference's pickled stage files to engine stage files, executing nothing.

The reference's offline splitter stores each span as a pickled nn.Module
(`torch.save(module, parts_dir/<name>/model.pth)`, split_model.py:107) that only
`torch.load(..., weights_only=False)` can read (partitioned_models.py:112-117), i.e. by
running whatever the pickle names.  This converter reads such a file with an inert
unpickler instead:
  * every class or function the pickle names becomes an inert stub (its constructor,
    __setstate__ and any call only record their arguments; no code of the named module is
    imported or run), except a closed list of tensor-rebuild helpers that are re-implemented
    here (`_rebuild_tensor_v2`, `_rebuild_parameter`, OrderedDict, storage dtype markers);
  * tensor storages are read from the zip archive's data/ records (persistent ids);
  * the module tree is walked through the recorded `_modules` / `_parameters` /
    `_buffers` states, which gives module.state_dict()'s keys: `embed.weight`,
    `layers.<j>.self_attn.q_proj.weight`, ..., `norm.weight`, `lm_head.weight`.
The span's weights are then written as the safetensors stage file inferd_amd.split_model
writes (same keys and metadata), which PartitionedQwen2 loads.

    python -m inferd_amd.convert_parts --config petals/inferd.yaml --model qwen3-0.6b \
        [--parts-dir model_parts] [--out converted_parts]
"""
from __future__ import annotations

import argparse
import os
import pickle
import zipfile
from collections import OrderedDict

import numpy as np
import torch

_STORAGE_DTYPES = {
    "FloatStorage": torch.float32, "BFloat16Storage": torch.bfloat16, "HalfStorage": torch.float16,
    "DoubleStorage": torch.float64, "LongStorage": torch.int64, "IntStorage": torch.int32,
    "BoolStorage": torch.bool, "ByteStorage": torch.uint8, "UntypedStorage": torch.uint8,
}
_DTYPE_NAMES = {"float32": torch.float32, "bfloat16": torch.bfloat16, "float16": torch.float16,
                "float64": torch.float64, "int64": torch.int64, "int32": torch.int32, "bool": torch.bool,
                "uint8": torch.uint8}


class Stub:
    """Inert stand-in for any class or function a pickle names: constructing it (NEWOBJ /
    REDUCE) and __setstate__ (BUILD) only record their arguments."""

    qualname = "?"

    def __new__(cls, *args, **kwargs):
        return object.__new__(cls)

    def __init__(self, *args, **kwargs):
        self.args, self.state = args, None

    def __setstate__(self, state):
        self.state = state

    def __repr__(self):
        return f"Stub({self.qualname})"


_STUBS: dict = {}


def _stub_class(qualname: str) -> type:
    if qualname not in _STUBS:
        _STUBS[qualname] = type("Stub_" + qualname.replace(".", "_"), (Stub,), {"qualname": qualname})
    return _STUBS[qualname]


class _StorageMarker:
    def __init__(self, dtype):
        self.dtype = dtype


def _rebuild_tensor_v2(storage, storage_offset, size, stride, requires_grad=False, backward_hooks=None,
                       metadata=None):
    return torch.as_strided(storage, tuple(size), tuple(stride), storage_offset)


def _rebuild_parameter(data, requires_grad=False, backward_hooks=None, *extra):
    return data


def _reconstructor(cls, base, state=None):
    """copyreg._reconstructor restricted to stubs."""
    if isinstance(cls, type) and issubclass(cls, Stub):
        return object.__new__(cls)
    raise pickle.UnpicklingError(f"refusing to reconstruct {cls!r}")


_BUILTINS = {"set": set, "frozenset": frozenset, "list": list, "dict": dict, "tuple": tuple, "object": object}


class InertUnpickler(pickle.Unpickler):
    def __init__(self, f, zf: zipfile.ZipFile, prefix: str):
        super().__init__(f)
        self.zf, self.prefix = zf, prefix

    def find_class(self, module, name):
        if module == "torch._utils" and name == "_rebuild_tensor_v2":
            return _rebuild_tensor_v2
        if module == "torch._utils" and name in ("_rebuild_parameter", "_rebuild_parameter_with_state"):
            return _rebuild_parameter
        if module == "collections" and name == "OrderedDict":
            return OrderedDict
        if module == "copyreg" and name == "_reconstructor":
            return _reconstructor
        if module in ("torch", "torch.storage") and name in _STORAGE_DTYPES:
            return _StorageMarker(_STORAGE_DTYPES[name])
        if module == "torch" and name in _DTYPE_NAMES:
            return _DTYPE_NAMES[name]
        if module in ("builtins", "__builtin__") and name in _BUILTINS:
            return _BUILTINS[name]
        return _stub_class(f"{module}.{name}")

    def persistent_load(self, pid):
        # ('storage', storage type, key, location, numel)
        if not (isinstance(pid, tuple) and pid and pid[0] == "storage"):
            raise pickle.UnpicklingError(f"unexpected persistent id {pid!r}")
        typ, key = pid[1], pid[2]
        dtype = typ.dtype if isinstance(typ, _StorageMarker) else (typ if isinstance(typ, torch.dtype) else torch.uint8)
        raw = self.zf.read(f"{self.prefix}data/{key}")
        if dtype == torch.bool:
            return torch.from_numpy(np.frombuffer(raw, dtype=np.uint8).copy()).to(torch.bool)
        return torch.frombuffer(bytearray(raw), dtype=dtype) if raw else torch.empty(0, dtype=dtype)


def load_inert(path: str):
    """The object tree of a torch.save zip archive, every named class replaced by a Stub."""
    with zipfile.ZipFile(path) as zf:
        pkl = [n for n in zf.namelist() if n.endswith("data.pkl")]
        if len(pkl) != 1:
            raise ValueError(f"{path}: not a torch.save zip archive")
        prefix = pkl[0][:-len("data.pkl")]
        import io
        return InertUnpickler(io.BytesIO(zf.read(pkl[0])), zf, prefix).load()


def module_state_dict(obj, prefix: str = "") -> dict:
    """module.state_dict() of a stubbed nn.Module tree (parameters and persistent buffers)."""
    out = {}
    st = obj.state if isinstance(obj, Stub) else None
    if not isinstance(st, dict):
        return out
    for name, t in (st.get("_parameters") or {}).items():
        if t is not None:
            out[prefix + name] = t
    nonpersistent = st.get("_non_persistent_buffers_set") or set()
    for name, t in (st.get("_buffers") or {}).items():
        if t is not None and name not in nonpersistent:
            out[prefix + name] = t
    for name, m in (st.get("_modules") or {}).items():
        if m is not None:
            out.update(module_state_dict(m, prefix + name + "."))
    return out


# keys of a reference stage module -> engine stage-file keys (inferd_amd/split_model.py)
_LAYER_LEAVES = ("self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
                 "self_attn.o_proj.weight", "self_attn.q_norm.weight", "self_attn.k_norm.weight",
                 "mlp.gate_proj.weight", "mlp.up_proj.weight", "mlp.down_proj.weight",
                 "input_layernorm.weight", "post_attention_layernorm.weight")


def stage_tensors(sd: dict) -> dict:
    """Pick the span's weights out of a stage module's state dict (rotary inv_freq and the
    like are recomputed by the engine); reject layouts the Qwen3 engine does not run."""
    out = {}
    for k, v in sd.items():
        if k in ("embed.weight", "norm.weight", "lm_head.weight"):
            out[k] = v
        elif k.startswith("layers."):
            _, j, leaf = k.split(".", 2)
            if leaf.endswith(".bias"):
                raise ValueError(f"{k}: biased projections (Qwen2 layers) are not a Qwen3 span")
            if leaf in _LAYER_LEAVES:
                out[k] = v
    if not any(k.startswith("layers.") for k in out) and not out:
        raise ValueError("no span weights found (expected embed/layers/norm/lm_head keys)")
    return out


def convert(cfg: dict, dims, parts_dir: str, out_dir: str) -> list:
    """One engine stage file per inferd.yaml entry, from parts_dir/<name>/model.pth."""
    from safetensors.torch import save_file
    import json
    from dataclasses import asdict
    n_stages = int(cfg["stages_count"])
    written = []
    for st in cfg["stages"]:
        src = os.path.join(parts_dir, st["name"], "model.pth")
        tensors = {k: v.to(torch.bfloat16).contiguous() for k, v in stage_tensors(module_state_dict(load_inert(src))).items()}
        stage = int(st["stage"])
        meta = {"dims": json.dumps(asdict(dims)), "start_layer": str(st["start_layer"]),
                "end_layer": str(st["end_layer"]), "first": "1" if stage == 0 else "0",
                "last": "1" if stage == n_stages - 1 else "0"}
        n_layers = int(st["end_layer"]) - int(st["start_layer"]) + 1
        have = {int(k.split(".")[1]) for k in tensors if k.startswith("layers.")}
        if have != set(range(n_layers)):
            raise ValueError(f"{src}: layers {sorted(have)} do not match start/end {st['start_layer']}-{st['end_layer']}")
        if meta["first"] == "1" and "embed.weight" not in tensors:
            raise ValueError(f"{src}: first stage without embed.weight")
        if meta["last"] == "1" and ("lm_head.weight" not in tensors or "norm.weight" not in tensors):
            raise ValueError(f"{src}: last stage without norm / lm_head")
        dst = os.path.join(out_dir, st["name"], "model.safetensors")
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        save_file(tensors, dst, metadata=meta)
        written.append(dst)
    return written


def main():
    import yaml
    from .runtime import MODELS
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", required=True, help="inferd.yaml-format span config")
    ap.add_argument("--model", required=True, help=f"model dims: one of {sorted(MODELS)}")
    ap.add_argument("--parts-dir", default=None, help="default: the config's parts_dir")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    with open(a.config) as f:
        cfg = yaml.safe_load(f)
    for p in convert(cfg, MODELS[a.model], a.parts_dir or cfg["parts_dir"], a.out):
        print("wrote", p)


if __name__ == "__main__":
    main()
