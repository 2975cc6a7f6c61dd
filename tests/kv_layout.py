"""Test helpers: decode the fragment-packed KV page layout of inferd_amd/csrc/common.h."""
import numpy as np
import torch

PAGE, D = 64, 128


def _k_index():
    idx = np.zeros((PAGE, D), dtype=np.int64)
    for tb in range(4):
        for ks in range(4):
            for l in range(64):
                for j in range(8):
                    idx[16 * tb + (l & 15), 32 * ks + 8 * (l >> 4) + j] = ((tb * 4 + ks) * 64 + l) * 8 + j
    return torch.from_numpy(idx)


def _vperm(g, j):
    return 4 * g + j if j < 4 else 16 + 4 * g + (j - 4)


def _v_index():
    idx = np.zeros((PAGE, D), dtype=np.int64)
    for kt in range(2):
        for db in range(8):
            for l in range(64):
                for j in range(8):
                    idx[32 * kt + _vperm(l >> 4, j), 16 * db + (l & 15)] = ((kt * 8 + db) * 64 + l) * 8 + j
    return torch.from_numpy(idx)


K_IDX, V_IDX = _k_index(), _v_index()


SUPER = 16  # pages per super-page (common.h KV_SUPER)


def pool_elems(pages: int, kv_heads: int) -> int:
    """bf16 elements of a pool holding `pages` pages, rounded up to whole super-pages."""
    return (pages + SUPER - 1) // SUPER * SUPER * 2 * kv_heads * PAGE * D


def block(kv_layer: torch.Tensor, kv_heads: int, page: int, kind: int) -> torch.Tensor:
    """(kv_heads, 64*128) view of page `page`'s K (kind 0) or V (kind 1) blocks: the pool is
    [page // 16][kv head][page % 16][K|V][64 x 128] (common.h kv_block)."""
    return kv_layer.view(-1, kv_heads, SUPER, 2, PAGE * D)[page // SUPER, :, page % SUPER, kind]


def read_kv(kv_layer: torch.Tensor, kv_heads: int, pages, n_tokens: int):
    """kv_layer: flat bf16 tensor of one layer's pool.  Returns K, V as (kv_heads, n_tokens, 128)."""
    ks, vs = [], []
    for p in pages:
        kb = block(kv_layer, kv_heads, p, 0).cpu()
        vb = block(kv_layer, kv_heads, p, 1).cpu()
        ks.append(kb[:, K_IDX.reshape(-1)].reshape(kv_heads, PAGE, D))
        vs.append(vb[:, V_IDX.reshape(-1)].reshape(kv_heads, PAGE, D))
    K = torch.cat(ks, dim=1)[:, :n_tokens]
    V = torch.cat(vs, dim=1)[:, :n_tokens]
    return K, V
