"""A 10M-resource config-4 sweep on one MI355X:
10M mixed objects (Pods, Deployments, Services, ConfigMaps, Namespaces) x 50
randomized constraints staged once and evaluated in one call, with the 64-bit
output cursors exercised (message bytes beyond 4 GiB), then parity on a
random sample of reviews: their rows are picked out of the device output on
the GPU (the raw gk_viol records + message bytes, flagged reviews already
dropped) and compared with the oracle's.

usage: python tools/sweep_10m.py [n=10000000] [sample=600]
prints one JSON line (also written to gpurun_out/sweep_10m.json)."""
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client, augmented_review  # noqa: E402
from gkgpu.driver import Result, Results  # noqa: E402
from gkgpu.page import Page  # noqa: E402
from gkgpu.parallel import DeviceOutput, unpack_viol  # noqa: E402
from parity import compare, oracle_for  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    n_sample = int(sys.argv[2]) if len(sys.argv) > 2 else 600
    out = {"resources": n, "sample": n_sample}
    ts, cs = W.config4()
    t0 = time.time()
    objs, nss = W.gen_config4_json(n, seed=2024)
    out["gen_s"] = round(time.time() - t0, 1)
    rng = random.Random(7)
    sample = sorted(rng.sample(range(n), n_sample))
    s_objs = [json.loads(objs[i]) for i in sample]
    s_nss = [None if nss[i] is None else json.loads(nss[i]) for i in sample]
    page = Page.from_lists(objs, nss)
    del objs, nss
    print("generated", out["gen_s"], "s", flush=True)

    drv = gkgpu.Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    t0 = time.time()
    batch = drv.stage_page(page)
    out["stage_s"] = round(time.time() - t0, 2)
    del page
    print("staged", out["stage_s"], "s", flush=True)
    dev = torch.device("cuda", 0)
    dout = DeviceOutput(dev)
    batch.eval(decode=False, light=True)  # warm-up: JIT + buffer sizing
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = batch.eval(decode=False, light=True, device_out=dout, with_status=True)
    torch.cuda.synchronize()
    out["eval_s"] = round(time.perf_counter() - t0, 3)
    out["evals"] = n * len(cs)
    out["device_tuples"] = res.device_tuples
    out["device_bytes"] = res.device_bytes
    out["bytes_beyond_4GiB"] = res.device_bytes > (1 << 32)
    out["kernel_ms"] = round(sum(ln.ms for ln in res.launches), 2) if hasattr(res, "launches") else None
    out["fallback_reviews"] = res.n_fallbacks
    out["error_reviews"] = res.n_errors
    out["copied_tuples"] = dout.n_tuples
    print("evaluated", out["eval_s"], "s", res.device_tuples, "tuples", res.device_bytes, "bytes", flush=True)

    # the sampled reviews' rows, picked on the GPU
    tup = dout.tuples()
    idx = torch.tensor(sample, dtype=torch.int32, device=dev)
    sel = tup[torch.isin(tup[:, 0], idx)].cpu().numpy()
    raw = dout.bytes()
    pos = {r: k for k, r in enumerate(sample)}
    cons = drv.constraints()
    ea = {(c["kind"], c["metadata"]["name"]): c.get("spec", {}).get("enforcementAction", "deny") for c in cs}
    rows = []
    for rec in sel:
        rv, c, seq, rule, ml, mo, dl = unpack_viol(rec)
        b = raw[mo:mo + ml + dl].cpu().numpy().tobytes()
        kind, name = cons[c]
        rows.append(Result(pos[rv], c, kind, name, b[:ml].decode("utf-8", "surrogateescape"),
                           b[ml:].decode("utf-8", "surrogateescape"), ea[(kind, name)]))
    status = [int(res.status[i]) if len(res.status) else 0 for i in sample]
    sub = Results(rows, status, [0] * n_sample, [])
    od = oracle_for(ts, cs)
    t0 = time.time()
    rep = compare(od, [augmented_review(o, s) for o, s in zip(s_objs, s_nss)], sub)
    out["oracle_s"] = round(time.time() - t0, 1)
    out["sample_report"] = repr(rep)
    out["sample_mismatches"] = len(rep.mismatches)
    out["sample_violations"] = rep.violations
    out["parity"] = not rep.mismatches and rep.compared > 0
    line = json.dumps(out)
    print(line, flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "sweep_10m.json"), "w") as f:
        f.write(line + "\n")
    if rep.mismatches:
        print(rep.mismatches[:3])
        sys.exit(1)


if __name__ == "__main__":
    main()
