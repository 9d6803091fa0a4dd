"""Per-wave phase timing of the u16 scan kernel (general maps) in the timing build
(build/xp/libblt_bpe_timing.so: tools/build_variant.sh timing -DBLT_TIMING), on the 256 MiB
multi-pass case of tools/config_rates.py (chained text map: one byte pass, one u16 pass).

    python tools/tok_timing.py [MiB]
Prints mean cycles per wave of: x-wait, phase 1, look-back + publish, look-back wait, emission,
ticket wait — of the first u16 pass (the records of later passes that return at once are empty)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("BLT_LIB_PATH", os.path.join(ROOT, "build", "exp", "libblt_bpe_timing.so"))
import torch  # noqa: E402

import blt_amd  # noqa: E402
from blt_amd import synth  # noqa: E402

TOK_TILE = 32768
CHUNK = 16 << 20
MAP = {(101, 32): 256, (256, 116): 257, (116, 104): 65, (65, 101): 258, (32, 116): 259, (259, 104): 260}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    s = blt_amd.BpeStrategy(MAP)
    data = synth.text(n, seed=2)
    d_in = torch.from_numpy(data).cuda()
    d_out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    wsb = s.workspace_size(n, CHUNK)
    ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
    nt_ws = (n + TOK_TILE - 1) // TOK_TILE
    tot_at = (64 + 8 * nt_ws + 15) // 16 * 16
    dbg = torch.zeros((8 + 8 * 16) * nt_ws + 64, dtype=torch.int64, device="cuda")
    L = blt_amd._lib.lib()
    L.blt_debug_set_tile_record.argtypes = [ctypes.c_void_p]
    sp = torch.cuda.current_stream().cuda_stream
    for it in range(3):
        dbg.zero_()
        L.blt_debug_set_tile_record(dbg.data_ptr() if it == 2 else None)
        s.encode_device(d_in.data_ptr(), n, CHUNK, d_out.data_ptr(), ws.data_ptr(), wsb, sp, sync=True)
    L.blt_debug_set_tile_record(None)
    tok0 = int(ws[tot_at:tot_at + 8].cpu().numpy().view(np.uint64)[0])   # byte-pass tokens
    ntiles = (tok0 + TOK_TILE - 1) // TOK_TILE
    print(f"byte-pass tokens {tok0}, u16 tiles {ntiles}, u16 passes {L.blt_debug_last_u16_passes()}")
    rec = dbg.cpu().numpy().astype(np.int64)
    wv = rec[8 * ntiles: 8 * ntiles + 8 * 16 * ntiles].reshape(ntiles, 16, 8)[:, :, :6]
    ok = wv[:, 0, :].sum(axis=1) > 0
    wv = wv[ok]
    names = ["x-wait", "phase1", "lb+pub", "lb-wait", "emit", "tk-wait"]
    print(f"{ok.sum()} tiles with records; per wave mean cycles: " + " ".join(f"{x:>8s}" for x in names) + "     total")
    for w in range(16):
        m = wv[:, w, :].mean(axis=0)
        print(f"  wave {w:2d}:          " + " ".join(f"{v:8.0f}" for v in m) + f"  {m.sum():8.0f}")


if __name__ == "__main__":
    main()
