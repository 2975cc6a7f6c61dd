"""Test fixtures in the on-disk formats the engine must ingest, built from the
oracle's counter-based weights so that the engine's result on them is known:
  * a HF-format safetensors checkpoint directory (two shards; keys model.layers.{i}.*,
    model.embed_tokens.weight, model.norm.weight, lm_head.weight), as split_model.py:81's
    from_pretrained source would hold;
  * the reference's pickled stage modules, parts_dir/<name>/model.pth = torch.save(module)
    of a module tree with the reference's attribute layout (split_model.py:13-70: embed /
    rotary / layers / norm / lm_head) over transformers' Qwen3DecoderLayer."""
import os

import torch
from torch import nn

from oracle import qwen3_ref as R

_ATTN = ("q_proj", "k_proj", "v_proj", "o_proj", "q_norm", "k_norm")


def layer_state_dict(d, seed, i):
    return {("self_attn." if k in _ATTN else "mlp." if k.endswith("_proj") else "") + k + ".weight": v
            for k, v in R.gen_layer_weights(d, seed, i).items()}


def write_hf_checkpoint(path, d, seed):
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    g = R.gen_global_weights(d, seed)
    shard0 = {"model.embed_tokens.weight": g["embed_tokens"]}
    shard1 = {"model.norm.weight": g["norm"], "lm_head.weight": g["lm_head"]}
    for i in range(d.layers):
        tgt = shard0 if i < d.layers // 2 else shard1
        for k, v in layer_state_dict(d, seed, i).items():
            tgt[f"model.layers.{i}.{k}"] = v.contiguous()
    save_file(shard0, os.path.join(path, "model-00001-of-00002.safetensors"))
    save_file(shard1, os.path.join(path, "model-00002-of-00002.safetensors"))
    return path


class FirstStage(nn.Module):
    def __init__(self, embed, rotary, layers):
        super().__init__()
        self.embed, self.rotary, self.layers = embed, rotary, nn.ModuleList(layers)


class StageInner(nn.Module):
    def __init__(self, rotary, layers):
        super().__init__()
        self.rotary, self.layers = rotary, nn.ModuleList(layers)


class LastStage(nn.Module):
    def __init__(self, rotary, layers, norm, lm_head):
        super().__init__()
        self.rotary, self.layers, self.norm, self.lm_head = rotary, nn.ModuleList(layers), norm, lm_head


def _hf_config(d):
    from transformers import Qwen3Config
    return Qwen3Config(hidden_size=d.hidden, intermediate_size=d.intermediate, num_attention_heads=d.heads,
                       num_key_value_heads=d.kv_heads, head_dim=d.head_dim, vocab_size=d.vocab,
                       num_hidden_layers=d.layers, rms_norm_eps=d.eps, rope_theta=d.rope_theta,
                       max_position_embeddings=d.max_positions)


def write_reference_parts(parts_dir, cfg, d, seed):
    """torch.save(stage module) per inferd.yaml entry, roles from `stage` (split_model.py:92-108)."""
    from transformers.models.qwen3.modeling_qwen3 import Qwen3DecoderLayer, Qwen3RMSNorm, Qwen3RotaryEmbedding
    hc = _hf_config(d)
    g = R.gen_global_weights(d, seed)
    n_stages = int(cfg["stages_count"])
    for st in cfg["stages"]:
        layers = []
        for i in range(int(st["start_layer"]), int(st["end_layer"]) + 1):
            L = Qwen3DecoderLayer(hc, i).to(torch.bfloat16)
            L.load_state_dict(layer_state_dict(d, seed, i))
            layers.append(L)
        rot = Qwen3RotaryEmbedding(hc)
        stage = int(st["stage"])
        if stage == 0:
            emb = nn.Embedding(d.vocab, d.hidden).to(torch.bfloat16)
            emb.weight.data.copy_(g["embed_tokens"])
            mod = FirstStage(emb, rot, layers)
        elif stage == n_stages - 1:
            norm = Qwen3RMSNorm(d.hidden, eps=d.eps).to(torch.bfloat16)
            norm.weight.data.copy_(g["norm"])
            head = nn.Linear(d.hidden, d.vocab, bias=False).to(torch.bfloat16)
            head.weight.data.copy_(g["lm_head"])
            mod = LastStage(rot, layers, norm, head)
        else:
            mod = StageInner(rot, layers)
        os.makedirs(os.path.join(parts_dir, st["name"]), exist_ok=True)
        torch.save(mod, os.path.join(parts_dir, st["name"], "model.pth"))
