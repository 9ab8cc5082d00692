"""PROBE TOOLING: which CUs a hipExtStreamCreateWithCUMask mask names
(tools/libstandin.so standin_whoami: 2048 one-wave blocks on a stream with
the mask, each reading HW_REG_XCC_ID and HW_REG_HW_ID).  Per mask: how many
distinct CUs the blocks ran on, per XCC.  One JSON line.

    python tools/cumask_map.py
"""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BLOCKS = 2048


def main():
    dev = torch.device("cuda", 0)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    nw = (ncu + 31) // 32
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libstandin.so"))
    lib.standin_whoami.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    out = torch.zeros(2 * BLOCKS, dtype=torch.int32, device=dev)

    def where(bits):
        words = (ctypes.c_uint32 * nw)()
        for i in bits:
            words[i // 32] |= 1 << (i % 32)
        out.zero_()
        assert lib.standin_whoami(nw, words, BLOCKS, out.data_ptr()) == 0
        v = out.view(BLOCKS, 2).cpu().tolist()
        return sorted({(x & 0xf, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 0xf) for x, h in v})

    def summary(bits):
        cus = where(bits)
        per = {}
        for c in cus:
            per[c[0]] = per.get(c[0], 0) + 1
        return {"cus": len(cus), "per_xcc": per}

    masks = {
        "all": range(ncu),
        "bit0": [0], "bit255": [ncu - 1], "bits0_1": [0, 1],
        "chunk0 (0-31)": range(32), "chunk7 (224-255)": range(ncu - 32, ncu),
        "half (0-127)": range(ncu // 2),
        "mod8==0": [j for j in range(ncu) if j % 8 == 0],
        "mod8!=7": [j for j in range(ncu) if j % 8 != 7],
        "mod32<28": [j for j in range(ncu) if j % 32 < 28],
        "mod32>=28": [j for j in range(ncu) if j % 32 >= 28],
        "lt224": range(ncu - 32),
    }
    # CU index c within each XCC = bit // 8: where does c sit (se, sh, cu)?
    per_c = {}
    for c in range(ncu // 8):
        cus = where(range(8 * c, 8 * c + 8))
        per_c[c] = sorted({(se, sh, cu) for _, se, sh, cu in cus})
    print(json.dumps({"ncu": ncu, "masks": {k: summary(v) for k, v in masks.items()},
                      "cu_index_to_se_sh_cu": per_c}))


if __name__ == "__main__":
    main()
