#!/usr/bin/env python3
"""Audit-sweep benchmark: resource x constraint evals/sec on MI355X.

Workload (BASELINE.json configs[1]): demo/agilebank policies (required labels,
allowed repos, container limits, required probes) over synthetic Pods,
1,000,000 Pods per GPU (weak scaling: each rank audits its own shard; the only
exchange step is the all-reduce of per-constraint violation totals the audit
status write needs, pkg/audit/manager.go:462-508, over RCCL).

A step = one audit sweep of the rank's staged (HBM-resident) batch: match +
template predicates + GPU message formatting + tuple compaction + totals
all-reduce.  Run as `python bench.py --gpus N --steps K --warmup W` (N>1 under
torch.distributed.run).  Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 20; 1000 launches for config 5)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="2", choices=sorted(CONFIGS),
                    help="BASELINE.json configs[n-1]: 2 = agilebank x Pods (the metric's config), "
                         "3 = allowedRegex x Deployments+Services, 4 = mixed kinds x 50 constraints (per-GPU shard), "
                         "5 = admission-webhook micro-batch (256 AdmissionReviews per launch, p50/p99 latency)")
    ap.add_argument("--load", type=int, default=50, help="config 5: constraints loaded (policy_benchmark_test.go:268)")
    ap.add_argument("--batch", type=int, default=256, help="config 5: AdmissionReviews per launch")
    ap.add_argument("--coalesce-us", type=int, default=0,
                    help="config 5: instead of pre-assembled batches, --clients threads issue single-review "
                         "Query calls at --rate requests/s (open loop) and the engine's micro-batch coalescer "
                         "gathers them for this many microseconds (up to --batch per launch); latency includes "
                         "the queueing")
    ap.add_argument("--clients", type=int, default=64, help="config 5 coalesced: concurrent client threads")
    ap.add_argument("--rate", type=float, default=20000.0, help="config 5 coalesced: offered requests/s (total)")
    ap.add_argument("--loadgen", choices=("native", "python"), default="native",
                    help="config 5: the timed calls from C++ (libgkload.so) or from Python")
    ap.add_argument("--pods", type=int, default=None, help="resources per GPU (default: the config's)")
    ap.add_argument("--cpu-sample", type=int, default=-1,
                    help="resources of the staged batch timed on the native CPU baseline (oracle/cpuvm.cc; "
                         "-1 = all of them, 0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = every core this process may run on: the CPU affinity set, "
                         "capped by a cgroup CPU quota when one is set)")
    ap.add_argument("--oracle-sample", type=int, default=0,
                    help="resources also timed on the Python oracle (1 core; 0 = skip)")
    ap.add_argument("--from-cache", action="store_true",
                    help="audit from the cache: the config's objects (and their Namespaces) synced into the "
                         "inventory with PutData, a step = one Client.Audit (hooks.audit) over all of them, every "
                         "result row decoded on the host (--audit-from-cache, manager.go:195-197)")
    ap.add_argument("--shard-leg", choices=("auto", "on", "off"), default="auto",
                    help="also time config 4's one-GPU shard (1.25M mixed resources x 50 constraints, the north "
                         "star's >=1M x 50 shape) in the same process and report it as `config4_shard` "
                         "(auto: on for config 2 at one GPU)")
    ap.add_argument("--cpu-e2e", choices=("on", "off"), default="on",
                    help="CPU baseline end to end: the port also parses and flattens the same page on the leased "
                         "cores before evaluating it (cpu_baseline.end_to_end)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per launch for this workload (rocprofv3 --pmc), if measured")
    return ap.parse_args()


# config -> (templates/constraints, JSON generator(n, start), default resources per GPU, description)
def _configs():
    from gkgpu import workloads as W
    return {
        "2": (W.config2, lambda n, start: W.gen_pods_json(n, seed=42, n_namespaces=1000, start=start), 1_000_000,
              "config2: demo/agilebank policies over synthetic Pods (BASELINE configs[1])"),
        "3": (W.config3, lambda n, start: W.gen_config3_json(n, seed=7, start=start), 1_000_000,
              "config3: 10 allowedRegex label/annotation constraints over Deployments + Services (BASELINE configs[2])"),
        "4": (W.config4, lambda n, start: W.gen_config4_json(n, seed=1234, start=start), 1_250_000,
              "config4: mixed kinds x 50 randomized constraints, 1.25M resources per GPU = 10M over 8 (BASELINE configs[3])"),
        "6": (W.config6, lambda n, start: W.gen_config6_json(n, start=start), 20_000,
              "config6: config 2's agilebank policies + demo/basic unique-label over synced Services and labelled "
              "Deployments, the same objects in data.inventory (the joins of VERDICT r02 next #6)"),
    }


def _inventory(config, gen, n):
    """config 6: the objects the audit reviews are also the synced inventory"""
    if config != "6":
        return []
    from gkgpu import workloads as W
    objs, _ = gen(n, 0)
    return W.inventory_paths(objs)


CONFIGS = ("2", "3", "4", "5", "6")


def spawn(args):
    """`--gpus N` without a launcher: start N rank processes under
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) before this
    process touches a GPU, and exit with their status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args))
    if args.config == "5":
        return webhook_main(args)
    if args.from_cache:
        return from_cache_main(args)
    if args.steps is None:
        args.steps = 20
    cfg_templates, cfg_gen, cfg_default_n, cfg_desc = _configs()[args.config]
    if args.pods is None:
        args.pods = cfg_default_n
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    xdev = "cuda"  # device of the exchange / timing tensors
    if world > 1:
        import torch
        import torch.distributed as dist  # noqa: F811
        # GKGPU_DIST_BACKEND=gloo: rehearsal of the multi-rank path on fewer
        # GPUs than ranks (ranks share devices round-robin; RCCL refuses two
        # ranks on one GPU), exchange tensors on the host.  Default: RCCL.
        backend = os.environ.get("GKGPU_DIST_BACKEND", "nccl")
        if backend == "gloo":
            local = local % max(1, torch.cuda.device_count())
            xdev = "cpu"
        torch.cuda.set_device(local)
        dist.init_process_group(backend)

    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client

    templates, constraints = cfg_templates()
    drv = gkgpu.Driver(device=local)
    cl = Client(drv)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    for path, obj in _inventory(args.config, cfg_gen, args.pods * world):
        drv.put_data(path, obj)
    n_cons = len(constraints)
    kinds = [t["spec"]["crd"]["spec"]["names"]["kind"] for t in templates]
    kinds_of = {}  # kernel name -> template kind
    for k in kinds:
        b, detail = drv.template_backend(k)
        if b == 2:
            kinds_of[detail] = k
        elif b == 3 and "[guard kernel " in detail:
            kinds_of[detail.split("[guard kernel ")[1].rstrip("]")] = k + " (guard)"

    from gkgpu.page import Page
    t0 = time.time()
    objs, nss = cfg_gen(args.pods, rank * args.pods)
    page = Page.from_lists(objs, nss)
    del objs, nss
    t_gen = time.time() - t0
    # the process's first HIP call initialises the runtime (~0.15 s, once per
    # process); a long-running audit process has paid it before any sweep
    t0 = time.time()
    gkgpu.Driver.device_available()
    t_devinit = time.time() - t0
    # templates and constraints compiled / uploaded before the sweep, as the
    # reference compiles at AddTemplate (timed apart: prepare_s)
    t0 = time.time()
    drv.prepare()
    t_prepare = time.time() - t0
    t0 = time.time()
    batch = drv.stage_page(page)
    t_stage = time.time() - t0
    stage_ms = batch.timing_ms()
    nrev, nodes, str_bytes, col_bytes = batch.stats()

    def sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()

    # stage time of the slowest rank (each rank flattens and uploads its shard)
    t_stage_max = t_stage
    if dist is not None:
        import torch
        t = torch.tensor([t_stage], dtype=torch.float64, device=xdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_stage_max = float(t.item())

    cons_ids = drv.constraints()
    base = rank * args.pods
    exch_ms = []
    writer = [None]

    def resource(i):
        _av, kind, name, ns = batch.resource(i)
        return kind, name, ns

    def step():
        # one audit sweep of the rank's shard: match + template predicates +
        # GPU message formatting + compaction + device-side status sampling
        # (exact totals, first 20 per constraint); then the exchange the audit
        # status needs: totals all-reduce + samples gathered to rank 0 over RCCL
        sweep = batch.eval_audit(limit=20)
        if dist is None:
            return sweep
        import torch
        from gkgpu.parallel import exchange_audit
        t0 = time.perf_counter()
        writer[0] = exchange_audit(sweep, base, resource, cons_ids, limit=20, dst=0,
                                   device=torch.device("cuda", local) if xdev == "cuda" else torch.device("cpu"))
        exch_ms.append((time.perf_counter() - t0) * 1000.0)
        return sweep

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    launch_ms = {}  # kernel name -> [ms per step]
    last = None
    for _ in range(args.steps):
        last = step()
        for ln in last.launches:
            launch_ms.setdefault(ln.kernel, []).append(ln.ms)
    sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=xdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1000.0
    # the core clock this box ran at, right after the timed region (box-to-box
    # variance of kernel times tracks it: DESIGN.md section 5)
    try:
        sclk_mhz = round(drv.debug_clock_mhz(), 1)
    except Exception:
        sclk_mhz = None
    evals_per_step = nrev * n_cons * world
    value = evals_per_step / (ms_per_step / 1000.0)
    # end to end: a cold sweep = flatten + H2D of the shard + one sweep (the
    # synthetic-input generation is excluded)
    e2e_s = t_stage_max + ms_per_step / 1000.0
    if writer[0] is None and rank == 0:
        from gkgpu.audit import AuditWriter
        from gkgpu.audit import FlaggedReviews
        try:
            writer[0] = AuditWriter.from_sweep(cons_ids, last, resource, 20)
        except FlaggedReviews:
            # flagged reviews would go to the CPU driver (reported below as
            # fallback_reviews / error_reviews); the bench has none to ask
            writer[0] = None
    status_totals = sum(writer[0].totals.values()) if writer[0] is not None else None

    # Roofline of the dominant kernel (the audit launch with the largest
    # average HIP-event duration).  Algorithmic bytes per launch follow SURVEY
    # 8(d): for the constraints the launch evaluates, 4 B per document value
    # the programs reference (an interned id, number id or row offset in a
    # columnar layout) + the bytes of the distinct strings whose bytes they
    # read + the match stage's id columns (kind, group, namespace: 12 B per
    # review) + 16 B per compacted violation tuple + 4 B per review of
    # error/fallback flags.  The references are counted by running the same
    # programs over the same staged batch in the CPU build of the device
    # runtime with its accounting hooks on (oracle/cpuvm_touch.cc).
    dom = max((k for k in launch_ms if k.startswith("gk_t_") or k == "audit_kernel"),
              key=lambda k: sum(launch_ms[k]))
    k_avg_ms = sum(launch_ms[dom]) / len(launch_ms[dom])
    dl = [ln for ln in last.launches if ln.kernel == dom][0]
    ref = referenced_bytes(drv, batch, kinds_of.get(dom), cons_ids, args.cpu_threads) if rank == 0 else None
    if ref is not None:
        algo_bytes = 4 * ref["nodes"] + ref["string_bytes"] + 12 * nrev + 16 * dl.tuples + 4 * nrev
    else:
        algo_bytes = None
    whole_store = nodes * 16 + str_bytes + col_bytes + dl.tuples * 32 + dl.bytes
    achieved = algo_bytes / (k_avg_ms / 1000.0) / 1e9 if algo_bytes else None
    # Sweep-level roofline (SURVEY 8(d)'s own definition: every referenced byte
    # counted ONCE per sweep, all constraints evaluated per resource): the union
    # of the document values every constraint references + their distinct
    # string bytes + the match id columns + 16 B per tuple of the whole sweep +
    # 4 B per review, over the whole step (ms_per_step: every kernel, the
    # format and sampling passes and the host work between them included)
    sweep_ref = referenced_bytes(drv, batch, None, cons_ids, args.cpu_threads, every=True) if rank == 0 else None
    sweep_bytes = None
    if sweep_ref is not None:
        sweep_bytes = 4 * sweep_ref["nodes"] + sweep_ref["string_bytes"] + 12 * nrev + 16 * last.device_tuples + 4 * nrev
    kernels = [{"kernel": ln.kernel, "avg_ms": sum(launch_ms[ln.kernel]) / len(launch_ms[ln.kernel]),
                "constraints": ln.constraints, "tuples": ln.tuples, "bytes": ln.bytes} for ln in last.launches]
    # the message format pass (gk_format_kernel): per tuple it reads the 32-B
    # tuple and its record (8-B header + 8 B per argument; 8 + 8*3 at most for
    # these templates, counted as 32 B) and writes the message bytes
    fmt_roof = None
    if "gk_format_kernel" in launch_ms:
        f_ms = sum(launch_ms["gk_format_kernel"]) / len(launch_ms["gk_format_kernel"])
        f_bytes = last.device_tuples * (32 + 32) + last.device_bytes
        f_ach = f_bytes / (f_ms / 1000.0) / 1e9
        f_tr = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("pods") == args.pods and tj.get("constraints") == n_cons:
                    f_tr = tj.get("hbm_bytes_per_launch", {}).get("gk_format_kernel")
            except Exception:
                f_tr = None
        fmt_roof = {"bound": "hbm", "achieved": f_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": f_ach / HBM_PEAK_GBS, "traffic": f_tr, "algo_bytes_per_launch": f_bytes,
                    "kernel_ms_avg": f_ms, "tuples": last.device_tuples}
    fallback = last.n_fallbacks
    errors = last.n_errors
    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get("pods") == args.pods and tj.get("constraints") == n_cons and tj.get("config", "2") == args.config:
                traffic = tj.get("hbm_bytes_per_launch", {}).get(kinds_of.get(dom))
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample != 0:
        n_cpu = nrev if args.cpu_sample < 0 else min(args.cpu_sample, nrev)
        cpu = native_cpu_baseline(drv, batch, n_cpu, args.cpu_threads, last)
        if args.cpu_e2e == "on" and n_cpu == nrev:
            # like for like with end_to_end_evals_per_s: the port parses and
            # flattens the same page on the same leased cores, then evaluates
            cpu["end_to_end"] = native_cpu_end_to_end(templates, constraints, page,
                                                      _inventory(args.config, cfg_gen, args.pods * world),
                                                      args.cpu_threads)
        if args.oracle_sample > 0:
            sample = page.slice(0, min(args.oracle_sample, page.n))
            so = [sample.objs[int(sample.obj_offs[i]):int(sample.obj_offs[i + 1])].decode() for i in range(sample.n)]
            sn = [None if k == 0xFFFFFFFF else page.nss[int(page.ns_offs[k]):int(page.ns_offs[k + 1])].decode()
                  for k in sample.obj_ns]
            cpu["python_oracle"] = cpu_baseline(templates, constraints, so, sn)

    if rank == 0:
        out = {
            "metric": "resource x constraint evals/sec (1/2/4/8 GPU) + % HBM roofline; vs host-CPU OPA",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded generator, SURVEY 8(d) config %s distribution)" % args.config,
            "config": {
                "workload": cfg_desc,
                "resources_per_gpu": nrev,
                "constraints": n_cons,
                "templates": [t["spec"]["crd"]["spec"]["names"]["kind"] for t in templates],
                "evals_per_step": evals_per_step,
                "violations_per_step_rank0": last.device_tuples,
                "excluded_reviews": last.excluded,
                "fallback_reviews": fallback,
                "error_reviews": errors,
                "parallelism": "dp%d (contiguous resource shards; per step: totals all-reduce (int64) + "
                               "first-20-per-constraint samples gathered to rank 0 over RCCL)" % world,
                "exchange_ms_avg_rank0": (sum(exch_ms[-args.steps:]) / args.steps) if exch_ms else 0.0,
                "status_total_violations": status_totals,
                "end_to_end_evals_per_s": evals_per_step / e2e_s,
                "end_to_end_s": e2e_s,
                "kernel_ms_per_step": sum(k["avg_ms"] for k in kernels),
                "kernel_only_evals_per_s": evals_per_step / (sum(k["avg_ms"] for k in kernels) / 1000.0),
                "backends": {k: {0: "cpu-fallback", 1: "bytecode-vm", 2: "template-kernel", 3: "guard-kernel+cpu-fallback"}[drv.template_backend(k)[0]]
                             for k in kinds},
                "kernel_templates": kinds_of,
                "sclk_mhz_measured": sclk_mhz,
                "device": device_info(local),
                "dist_backend": (os.environ.get("GKGPU_DIST_BACKEND", "nccl") if dist is not None else None),
                "stage_s": round(t_stage, 3),
                "stage_s_max_over_ranks": round(t_stage_max, 3),
                # host -> device bytes of the staged batch (16-B document nodes
                # + 48-B review columns; the shared string table is uploaded
                # separately and grows only by the page's new strings)
                "upload_bytes": batch.device_bytes(),
                "upload_bytes_per_resource": round(batch.device_bytes() / max(1, nrev), 1),
                "stage_ms": {"parse": round(stage_ms[0], 1), "flatten": round(stage_ms[1], 1),
                             "upload": round(stage_ms[2], 1)},
                "gen_s": round(t_gen, 3),
                "device_init_s": round(t_devinit, 3),
                "prepare_s": round(t_prepare, 3),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": traffic,
                "algo_bytes_per_launch": algo_bytes,
                "algo_bytes_definition": "SURVEY 8(d): 4 B x referenced document values + distinct string bytes "
                                         "read + 12 B x reviews (match id columns) + 16 B x tuples + 4 B x reviews",
                "referenced": ref,
                "whole_store_bytes_per_launch": whole_store,
                "whole_store_frac": whole_store / (k_avg_ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
                "kernel_ms_avg": k_avg_ms,
                "kernel": dom,
                "template": kinds_of.get(dom),
                "sweep_algo_bytes": sweep_bytes,
                "sweep_achieved": (sweep_bytes / (ms_per_step / 1000.0) / 1e9) if sweep_bytes else None,
                "sweep_frac": (sweep_bytes / (ms_per_step / 1000.0) / 1e9 / HBM_PEAK_GBS) if sweep_bytes else None,
                "sweep_definition": "SURVEY 8(d) per sweep: 4 B x the union of document values all constraints reference "
                                    "+ their distinct string bytes + 16 B x all tuples + 16 B x reviews, over ms_per_step",
            },
            "kernels": kernels,
            "format_pass": fmt_roof,
            "cpu_baseline": cpu,
            "config4_shard": None,
        }
        if world == 1 and (args.shard_leg == "on" or (args.shard_leg == "auto" and args.config == "2")):
            # the north star's shape (>=1M resources x 50 constraints): config
            # 4's one-GPU shard, timed in this process after the headline's
            # sweeps (its own engine; this one's device memory released first)
            batch.free()
            drv.close()
            out["config4_shard"] = shard_leg("4", 5, 1, args.cpu_threads)
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def shard_leg(cfg, steps, warmup, cpu_threads):
    """One configuration's one-GPU shard timed in the calling process (the
    headline line's `config4_shard`): staged once, `steps` audit sweeps after
    `warmup`, with its dominant kernel's roofline (SURVEY 8(d) algorithmic
    bytes over its HIP-event time) and the counts that make it comparable
    (fallback / error reviews, tuples)."""
    import gkgpu
    from gkgpu.client import Client
    from gkgpu.page import Page
    tfn, gen, n, desc = _configs()[cfg]
    templates, constraints = tfn()
    drv = gkgpu.Driver()
    cl = Client(drv)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    kinds_of = {}
    for t in templates:
        k = t["spec"]["crd"]["spec"]["names"]["kind"]
        b, detail = drv.template_backend(k)
        if b == 2:
            kinds_of[detail] = k
        elif b == 3 and "[guard kernel " in detail:
            kinds_of[detail.split("[guard kernel ")[1].rstrip("]")] = k + " (guard)"
    t0 = time.time()
    objs, nss = gen(n, 0)
    page = Page.from_lists(objs, nss)
    del objs, nss
    t_gen = time.time() - t0
    drv.prepare()
    t0 = time.time()
    batch = drv.stage_page(page)
    t_stage = time.time() - t0
    nrev = batch.stats()[0]
    for _ in range(warmup):
        batch.eval_audit(limit=20)
    launch_ms = {}
    t0 = time.perf_counter()
    last = None
    for _ in range(steps):
        last = batch.eval_audit(limit=20)
        for ln in last.launches:
            launch_ms.setdefault(ln.kernel, []).append(ln.ms)
    elapsed = time.perf_counter() - t0
    ms = elapsed / steps * 1000.0
    n_cons = len(constraints)
    dom = max((k for k in launch_ms if k.startswith("gk_t_") or k == "audit_kernel"), key=lambda k: sum(launch_ms[k]))
    k_ms = sum(launch_ms[dom]) / len(launch_ms[dom])
    dl = [ln for ln in last.launches if ln.kernel == dom][0]
    ref = referenced_bytes(drv, batch, kinds_of.get(dom), drv.constraints(), cpu_threads)
    algo = 4 * ref["nodes"] + ref["string_bytes"] + 12 * nrev + 16 * dl.tuples + 4 * nrev if ref else None
    ach = algo / (k_ms / 1000.0) / 1e9 if algo else None
    out = {
        "workload": desc,
        "resources": nrev,
        "constraints": n_cons,
        "value": nrev * n_cons / (ms / 1000.0),
        "unit": "evals/s",
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": ms,
        "timed_region_s": elapsed,
        "stage_s": round(t_stage, 3),
        "gen_s": round(t_gen, 3),
        "end_to_end_evals_per_s": nrev * n_cons / (t_stage + ms / 1000.0),
        "violations_per_step": last.device_tuples,
        "fallback_reviews": last.n_fallbacks,
        "error_reviews": last.n_errors,
        "kernel_ms_per_step": sum(sum(v) / len(v) for v in launch_ms.values()),
        "roofline": {"bound": "hbm", "kernel": dom, "template": kinds_of.get(dom), "kernel_ms_avg": k_ms,
                     "algo_bytes_per_launch": algo, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS if ach else None},
        "kernels": {kinds_of.get(k, k): round(sum(v) / len(v), 4) for k, v in launch_ms.items()},
    }
    batch.free()
    drv.close()
    return out


def native_cpu_end_to_end(templates, constraints, page, inventory, threads):
    """cpu_baseline.end_to_end: the port (oracle/cpuvm.cc, NOT OPA) timed like
    the GPU's end_to_end_evals_per_s -- the same page's JSON parsed and
    flattened by the engine's parallel flattener on the leased cores (a
    host-only engine), then every review x constraint evaluated on them."""
    import gkgpu
    from gkgpu.client import Client
    from oracle import cpu_baseline as CB
    hc = host_cpus()
    threads = threads or hc["lease"]
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    for path, obj in inventory:
        d.put_data(path, obj)
    d.template_backend(templates[0]["spec"]["crd"]["spec"]["names"]["kind"])  # compile before the clock
    # the per-document layout: the path-grouped one exists for the GPU's
    # coalesced wavefront reads and would only add host placement work here
    saved = os.environ.get("GKGPU_PATH_LAYOUT")
    os.environ["GKGPU_PATH_LAYOUT"] = "0"
    try:
        t0 = time.perf_counter()
        b = d.stage_page(page)
        stage_s = time.perf_counter() - t0
    finally:
        if saved is None:
            os.environ.pop("GKGPU_PATH_LAYOUT", None)
        else:
            os.environ["GKGPU_PATH_LAYOUT"] = saved
    secs, evals, viol, mbytes, flagged = CB.sweep(d, b, threads=threads)
    b.free()
    d.close()
    return {"value": evals / (stage_s + secs), "unit": "evals/s", "cores": threads, "kind": "port",
            "stage_seconds": stage_s, "eval_seconds": secs, "violations": viol, "flagged_pairs": flagged,
            "sample": "the same %d resources x %d constraints: JSON parse + flatten (engine flattener, host-only) "
                      "then oracle/cpuvm.cc evaluation, on %d threads; NOT OPA" % (evals // max(1, len(constraints)),
                                                                                  len(constraints), threads)}


def from_cache_main(args):
    """--from-cache (one GPU): Client.Audit over the synced inventory.  The
    engine keeps the inventory as a device-resident staged batch of
    make_review documents (target_template_source.go:46-89), built by the first
    audit after a change; every step evaluates it and decodes all result rows
    (Client.Audit returns every result, client.go:805-833)."""
    import re
    import gkgpu
    from gkgpu.client import Client, TARGET
    if args.steps is None:
        args.steps = 5
    cfg_templates, cfg_gen, cfg_default_n, cfg_desc = _configs()[args.config]
    n = args.pods or cfg_default_n
    templates, constraints = cfg_templates()
    drv = gkgpu.Driver()
    cl = Client(drv)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    objs, nss = cfg_gen(n, 0)
    t0 = time.time()
    ident = re.compile(r'\{"apiVersion":"([^"]*)","kind":"([^"]*)","metadata":\{"name":"([^"]*)"(?:,"namespace":"([^"]*)")?')
    seen_ns = set()
    for js, ns in zip(objs, nss):
        if ns is not None and id(ns) not in seen_ns:
            seen_ns.add(id(ns))
            nm = json.loads(ns)["metadata"]["name"]
            drv.put_data("/external/%s/cluster/v1/Namespace/%s" % (TARGET, nm), ns)
        m = ident.match(js)
        if m:
            av, kind, name, ons = m.group(1), m.group(2), m.group(3), m.group(4)
        else:  # another member order: read the identity from the parsed object
            o = json.loads(js)
            md = o.get("metadata") or {}
            av, kind, name, ons = o.get("apiVersion", ""), o.get("kind", ""), md.get("name", ""), md.get("namespace")
        gv = av.replace("/", "%2F")
        path = ("/external/%s/namespace/%s/%s/%s/%s" % (TARGET, ons, gv, kind, name) if ons
                else "/external/%s/cluster/%s/%s/%s" % (TARGET, gv, kind, name))
        drv.put_data(path, js)
    t_sync = time.time() - t0
    del objs, nss
    # a step = one --audit-from-cache sweep as the audit manager consumes it
    # (manager.go:195-207 then :462-508): Client.Audit over the synced
    # inventory reduced on the device to exact totals + the first 20 results
    # per constraint (gk_audit_cache_sample)
    t0 = time.perf_counter()
    first = drv.audit_sample(limit=20)
    t_first = time.perf_counter() - t0
    for _ in range(args.warmup):
        drv.audit_sample(limit=20)
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = drv.audit_sample(limit=20)
    elapsed = time.perf_counter() - t0
    # for reference: the same audit with every result row decoded on the host
    # (gk_query(hooks.audit), what Client.Audit returns)
    t0 = time.perf_counter()
    full = drv.audit_summary()
    full_ms = (time.perf_counter() - t0) * 1000.0
    builds, reviews = drv.audit_cache_stats()
    n_cons = len(constraints)
    ms = elapsed / args.steps * 1000.0
    out = {
        "metric": "resource x constraint evals/sec (1/2/4/8 GPU) + % HBM roofline; vs host-CPU OPA",
        "value": reviews * n_cons / (ms / 1000.0),
        "unit": "evals/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded generator, SURVEY 8(d) config %s distribution), synced with PutData" % args.config,
        "config": {
            "workload": cfg_desc + " -- audit from the cache (hooks.audit over the synced inventory)",
            "reviews": reviews,
            "constraints": n_cons,
            "results_per_audit": last.device_tuples,
            "status_totals": sum(last.totals),
            "samples": len(last.samples),
            "flagged_reviews": len(last.flagged),
            "cache_builds": builds,
            "first_audit_s": round(t_first, 3),
            "first_audit_timing_ms": [round(x, 2) for x in first.timing_ms],
            "steady_timing_ms": [round(x, 2) for x in last.timing_ms],
            "steady_launches": [(k.kernel, round(k.ms, 3), k.tuples) for k in last.launches],
            "timing_fields": "flatten, upload, kernels, download, decode (engine phases of one call)",
            "decode_all_rows_ms": round(full_ms, 2),
            "decode_all_rows_results": full["results"],
            "sync_s": round(t_sync, 1),
        },
        "roofline": None,
        "cpu_baseline": None,
    }
    print(json.dumps(out))


def referenced_bytes(drv, batch, kind, cons_ids, threads, every=False):
    """SURVEY 8(d) reference accounting of the constraints of template `kind`
    over the whole staged batch (oracle/cpuvm_touch.cc), or None; every=True:
    all constraints at once (a value several constraints read counts once)"""
    if every:
        sys.path.insert(0, ROOT)
        try:
            from oracle import cpu_baseline as CB
        except Exception:
            return None
        r = CB.referenced(drv, batch, -1, threads=threads if threads > 0 else host_cpus()["lease"])
        r["constraints"] = [n for _k, n in cons_ids]
        return r
    if kind is None:
        return None
    kind = kind.replace(" (guard)", "")
    sys.path.insert(0, ROOT)
    try:
        from oracle import cpu_baseline as CB
    except Exception:
        return None
    if threads <= 0:
        threads = host_cpus()["lease"]
    tot = {"nodes": 0, "strings": 0, "string_bytes": 0, "violations": 0, "flagged": 0, "constraints": []}
    for c, (k, name) in enumerate(cons_ids):
        if k != kind:
            continue
        r = CB.referenced(drv, batch, c, threads=threads)
        for f in ("nodes", "strings", "string_bytes", "violations", "flagged"):
            tot[f] += r[f]
        tot["constraints"].append(name)
    return tot


def device_info(dev):
    """the GPU the bench ran on: CU count (partition mode), memory, L2"""
    try:
        import torch
        p = torch.cuda.get_device_properties(dev)
        return {"name": p.name, "arch": getattr(p, "gcnArchName", None), "cus": p.multi_processor_count,
                "memory_gib": round(p.total_memory / 2**30, 1), "l2_bytes": getattr(p, "L2_cache_size", None)}
    except Exception:
        return None


def host_cpus():
    """the host cores this process is leased: nproc (os.cpu_count), the CPU
    affinity set, and a cgroup CPU quota (v2 cpu.max or v1 cfs quota/period)
    if one is set; `lease` = the affinity set, capped by the quota"""
    import math
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    lease = min(aff, max(1, math.ceil(quota))) if quota else aff
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "lease": lease}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def native_cpu_baseline(drv, batch, n_cpu, threads, gpu_sweep):
    """The native CPU baseline (oracle/cpuvm.cc): the engine's compiled
    template bytecode and device runtime, built for the host, over the first
    `n_cpu` reviews of the same staged batch x every constraint on `threads`
    host threads (messages formatted).  NOT OPA: Go/OPA v0.21 cannot be built
    offline; this is a far leaner CPU evaluator than the
    reference's per-Review topdown + JSON round trips."""
    sys.path.insert(0, ROOT)
    from oracle import cpu_baseline as CB
    hc = host_cpus()
    if threads <= 0:
        threads = hc["lease"]
    secs, evals, viol, mbytes, flagged = CB.sweep(drv, batch, 0, n_cpu, threads)
    out = {"value": evals / secs, "unit": "evals/s", "cores": threads, "kind": "port", "host_cpus": hc,
           "sample": "%d resources x %d constraints of the same staged batch (%s); oracle/cpuvm.cc: the engine's "
                     "compiled bytecode + device runtime on host threads, NOT OPA (Go/OPA not buildable offline)"
                     % (n_cpu, len(gpu_sweep.totals), "all" if n_cpu == batch.n else "prefix"),
           "seconds": secs, "cpu_model": cpu_model(), "violations": viol, "message_bytes": mbytes,
           "flagged_pairs": flagged}
    if n_cpu == batch.n:
        out["violations_equal_gpu"] = viol == gpu_sweep.device_tuples
    return out


def cpu_baseline(templates, constraints, objs_json, nss_json):
    """The oracle (CPU restatement of OPA topdown + the match library) timed on a
    bounded sample of the same workload, one core."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from parity import oracle_for, oracle_review
    from gkgpu.client import augmented_review
    od = oracle_for(templates, constraints)
    objs = [json.loads(o) for o in objs_json]
    nss = [None if n is None else json.loads(n) for n in nss_json]
    t0 = time.perf_counter()
    for o, n in zip(objs, nss):
        oracle_review(od, augmented_review(o, n))
    dt = time.perf_counter() - t0
    return {"value": len(objs) * len(constraints) / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": "%d resources x %d constraints (same workload), oracle/ CPU restatement of OPA v0.21 "
                      "topdown; Go/OPA not buildable offline" % (len(objs), len(constraints)),
            "seconds": dt}


def webhook_main(args):
    """Config 5 (BASELINE configs[4]): admission-webhook micro-batch.  A step is
    one gk_query_batch launch over `--batch` UPDATE AdmissionReviews (object +
    oldObject, policy_benchmark_test.go:197-231) against the PSP policies at
    constraint load `--load`, timed from the call's entry to decoded results
    (messages, details, enforcementAction) back on the host.  Inputs are JSON
    text (what the webhook receives), generated before the timed region."""
    if args.steps is None:
        args.steps = 1000
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist  # noqa: F811
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client
    from gkgpu.webhook import handle_batch  # noqa: F401  (the per-request decision path tests use)

    templates, constraints = W.config5(args.load)
    drv = gkgpu.Driver(device=local, coalesce_us=args.coalesce_us, coalesce_max=args.batch)
    cl = Client(drv)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    nb = 16
    batches = [W.gen_admission_inputs(args.batch, seed=99, start=(rank * nb + i) * args.batch) for i in range(nb)]
    for i in range(args.warmup):
        drv.query_batch(batches[i % nb])
    if dist is not None:
        dist.barrier()
    if args.coalesce_us:
        return webhook_coalesced_main(args, drv, templates, constraints, batches, world, rank, dist)
    # Timed: the C-ABI call (parse, flatten, upload, kernels, download,
    # decode) and one bulk copy of every decoded row (message, details) plus
    # the per-review status words into this process (gk_results_export), as a
    # native webhook caller reads them; building Python result objects is the
    # test harness's work and stays outside.
    lat = []
    n_results = n_flagged = 0
    blob_bytes = 0
    if args.loadgen == "native":
        # the same calls from C++ (gatekeeper-1_amd/csrc/loadgen.cc
        # gkload_batch_loop): the request bytes as the webhook receives them,
        # no Python marshalling inside the timed calls
        import ctypes as C
        lib = C.CDLL(os.path.join(ROOT, "gatekeeper-1_amd", "gkgpu", "libgkload.so"))
        lib.gkload_batch_loop.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t,
                                          C.c_size_t, C.c_size_t, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        blobs = [(x if isinstance(x, str) else json.dumps(x)).encode() for b in batches for x in b]
        arr = (C.c_char_p * len(blobs))(*blobs)
        lens = (C.c_size_t * len(blobs))(*[len(b) for b in blobs])
        lt = (C.c_double * args.steps)()
        rows, nbytes, nfl = C.c_uint64(), C.c_uint64(), C.c_uint64()
        t0 = time.perf_counter()
        rc = lib.gkload_batch_loop(drv._e, arr, lens, nb, args.batch, args.steps, lt, C.byref(rows), C.byref(nbytes),
                                   C.byref(nfl))
        elapsed = time.perf_counter() - t0
        if rc:
            raise RuntimeError("gkload_batch_loop: gk status %d" % rc)
        lat = list(lt)
        blob_bytes, n_flagged, n_results = nbytes.value, nfl.value, rows.value
    else:
        t0 = time.perf_counter()
        for i in range(args.steps):
            ts = time.perf_counter()
            blob, st = drv.query_batch_export(batches[i % nb])
            lat.append((time.perf_counter() - ts) * 1000.0)
            blob_bytes += len(blob)
            n_flagged += sum(1 for x in st if x & 3)
        elapsed = time.perf_counter() - t0
    res = drv.query_batch(batches[(args.steps - 1) % nb])
    if args.loadgen != "native":
        n_results = len(res.results) * args.steps
    kernel_ms = [ln.ms for ln in res.launches]
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    lat.sort()

    def pct(p):
        return lat[min(len(lat) - 1, int(round(p / 100.0 * (len(lat) - 1))))]

    n_cons = len(constraints)
    evals = args.steps * args.batch * n_cons * world
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample != 0:
        cpu = webhook_native_cpu_baseline(templates, constraints, batches, args.cpu_threads)
        if args.oracle_sample > 0:
            cpu["python_oracle"] = webhook_cpu_baseline(templates, constraints,
                                                        batches[0][: min(args.batch, args.oracle_sample)])
    if rank == 0:
        out = {
            "metric": "resource x constraint evals/sec (1/2/4/8 GPU) + % HBM roofline; vs host-CPU OPA",
            "value": evals / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1000.0,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (PSP pods of policy_benchmark_test.go as UPDATE AdmissionReviews, seed 99)",
            "config": {
                "workload": "config5: admission-webhook micro-batch, %d AdmissionReviews per launch x %d PSP "
                            "constraints (BASELINE configs[4])" % (args.batch, n_cons),
                "requests_per_launch": args.batch,
                "constraints": n_cons,
                "latency_ms": {"p50": pct(50), "p99": pct(99), "mean": sum(lat) / len(lat), "max": lat[-1]},
                "requests_per_s": args.steps * args.batch * world / elapsed,
                "results_per_launch": n_results / args.steps,
                "result_bytes_per_launch": blob_bytes / args.steps,
                "timed": "gk_query_batch + gk_results_export (one bulk copy of the decoded rows) + status words, "
                         + ("called from C++ (gatekeeper-1_amd/csrc/loadgen.cc gkload_batch_loop)"
                            if args.loadgen == "native" else "called from Python (ctypes)"),
                "flagged_reviews": n_flagged,
                "kernel_ms_last_launch": kernel_ms,
                "parallelism": "replicas%d (independent webhook replicas, no collective)" % world,
            },
            "roofline": None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def webhook_coalesced_main(args, drv, templates, constraints, batches, world, rank, dist):
    inputs = [x for b in batches for x in b]
    lat, elapsed, n, launches, served = webhook_coalesced(args, drv, inputs, len(constraints))
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    def pct(p):
        return lat[min(len(lat) - 1, int(round(p / 100.0 * (len(lat) - 1))))]
    n_cons = len(constraints)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample != 0:
        cpu = webhook_native_cpu_baseline(templates, constraints, batches, args.cpu_threads)
    if rank == 0:
        out = {
            "metric": "resource x constraint evals/sec (1/2/4/8 GPU) + % HBM roofline; vs host-CPU OPA",
            "value": n * n_cons * world / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1000.0,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (PSP pods of policy_benchmark_test.go as UPDATE AdmissionReviews, seed 99)",
            "config": {
                "workload": "config5 coalesced: single-review Query calls from %d client threads at %.0f req/s "
                            "offered (open loop), micro-batch coalescer window %d us / max %d, x %d PSP "
                            "constraints (BASELINE configs[4])" % (args.clients, args.rate, args.coalesce_us,
                                                                  args.batch, n_cons),
                "requests": n,
                "constraints": n_cons,
                "offered_requests_per_s": args.rate,
                "requests_per_s": n * world / elapsed,
                "latency_ms": {"p50": pct(50), "p99": pct(99), "mean": sum(lat) / len(lat), "max": lat[-1]},
                "latency_definition": "scheduled arrival -> the caller's rows back on the host (gk_query + "
                                      "gk_results_export), queueing included",
                "launches": launches,
                "mean_requests_per_launch": served / max(1, launches),
                "clients": "%s threads (%s)" % (args.clients, "native, gatekeeper-1_amd/csrc/loadgen.cc"
                                                if args.loadgen == "native" else "Python"),
                "parallelism": "replicas%d (independent webhook replicas, no collective)" % world,
            },
            "roofline": None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.destroy_process_group()


def webhook_native_cpu_baseline(templates, constraints, batches, threads):
    """oracle/cpuvm.cc (the engine's compiled bytecode + device runtime built
    for the host, NOT OPA) on host threads over the same AdmissionReviews,
    staged on the host: evals/s of the micro-batches' requests x constraints."""
    import gkgpu
    from gkgpu.client import Client
    from oracle import cpu_baseline as CB
    hc = host_cpus()
    threads = threads or hc["lease"]
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    inputs = [x for b in batches for x in b]
    # the port parses and flattens the requests' JSON as the GPU path does
    # (the engine's parallel flattener, micro-batch by micro-batch), then
    # evaluates them: `value` counts both, as the GPU latency does
    stage_s = 0.0
    for bt in batches:
        t0 = time.perf_counter()
        sb = d.debug_stage_inputs(bt)
        stage_s += time.perf_counter() - t0
        sb.free()
    b = d.debug_stage_inputs(inputs)
    secs, evals, viol, mbytes, flagged = CB.sweep(d, b, threads=threads)
    b.free()
    d.close()
    return {"value": evals / (secs + stage_s), "unit": "evals/s", "cores": threads, "kind": "port", "host_cpus": hc,
            "value_eval_only": evals / secs, "stage_seconds": stage_s,
            "sample": "%d AdmissionReviews (the benchmark's %d micro-batches) x %d constraints; request JSON parsed and "
                      "flattened per micro-batch, then oracle/cpuvm.cc: the engine's compiled bytecode + device runtime "
                      "on host threads, NOT OPA (Go/OPA not buildable offline)" % (len(inputs), len(batches),
                                                                                   len(constraints)),
            "seconds": secs + stage_s, "violations": viol, "message_bytes": mbytes, "flagged_pairs": flagged,
            "cpu_model": cpu_model()}


def webhook_coalesced(args, drv, inputs, n_cons):
    """Open-loop arrivals: `--clients` threads issue single-review
    Query(violation) calls (the reference webhook's one Review per request,
    pkg/webhook/policy.go:371-387) at `--rate` requests/s in total; the engine
    coalesces concurrent calls (include/gkgpu.h coalesce_us).  A request's
    latency runs from its scheduled arrival to its results back on the host,
    so it includes the time spent queued behind a busy client or launch."""
    import threading
    viol = 'hooks["admission.k8s.gatekeeper.sh"].violation'
    n = args.steps * args.batch  # requests
    if args.loadgen == "native":
        return webhook_coalesced_native(args, drv, inputs, viol, n)
    per = [n // args.clients + (1 if c < n % args.clients else 0) for c in range(args.clients)]
    gap = args.clients / args.rate  # each client's inter-arrival time
    lat = [[] for _ in range(args.clients)]
    errs = []
    start = [0.0]
    go = threading.Barrier(args.clients + 1)
    blobs = [b.encode() if isinstance(b, str) else b for b in inputs]

    def client(c):
        try:
            go.wait()
            t0 = start[0] + c * gap / args.clients
            for k in range(per[c]):
                due = t0 + k * gap
                now = time.perf_counter()
                if due > now:
                    time.sleep(due - now)
                drv.query_export(viol, blobs[(c + k * args.clients) % len(blobs)])
                lat[c].append((time.perf_counter() - due) * 1000.0)
        except Exception as ex:  # noqa: BLE001
            errs.append(repr(ex))
    th = [threading.Thread(target=client, args=(c,)) for c in range(args.clients)]
    for t in th:
        t.start()
    b0, r0 = drv.coalesce_stats()
    start[0] = time.perf_counter() + 0.05
    go.wait()
    for t in th:
        t.join()
    elapsed = time.perf_counter() - start[0]
    if errs:
        raise RuntimeError(errs[0])
    b1, r1 = drv.coalesce_stats()
    all_lat = sorted(x for l in lat for x in l)
    return all_lat, elapsed, n, b1 - b0, r1 - r0


def webhook_coalesced_native(args, drv, inputs, viol, n):
    """As webhook_coalesced, the clients being native threads of
    libgkload.so (gatekeeper-1_amd/csrc/loadgen.cc), C-ABI callers of gk_query
    + gk_results_export: Python client threads serialize on the interpreter
    lock and their tail, not the engine's, dominated the latency."""
    import ctypes as C
    lib = C.CDLL(os.path.join(ROOT, "gatekeeper-1_amd", "gkgpu", "libgkload.so"))
    lib.gkload_open_loop.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t,
                                     C.c_size_t, C.c_int, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    blobs = [b.encode() if isinstance(b, str) else b for b in inputs]
    arr = (C.c_char_p * len(blobs))(*blobs)
    lens = (C.c_size_t * len(blobs))(*[len(b) for b in blobs])
    lat = (C.c_double * n)()
    el = C.c_double()
    b0, r0 = drv.coalesce_stats()
    rc = lib.gkload_open_loop(drv._e, viol.encode(), arr, lens, len(blobs), n, args.clients, args.rate, lat, C.byref(el))
    if rc:
        raise RuntimeError("gkload_open_loop: gk status %d" % rc)
    b1, r1 = drv.coalesce_stats()
    return sorted(lat), el.value, n, b1 - b0, r1 - r0


def webhook_cpu_baseline(templates, constraints, inputs):
    """The oracle on one host core over one micro-batch of the same requests:
    per-request Query latency (the reference webhook evaluates one request per
    Review call, policy.go:371-387)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from parity import oracle_for, oracle_review
    od = oracle_for(templates, constraints)
    reviews = [json.loads(s)["review"] for s in inputs]
    lat = []
    for rv in reviews:
        t0 = time.perf_counter()
        oracle_review(od, rv)
        lat.append((time.perf_counter() - t0) * 1000.0)
    lat.sort()
    tot = sum(lat) / 1000.0
    return {"value": len(reviews) * len(constraints) / tot, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": "%d AdmissionReviews x %d constraints, one Query per request, oracle/ CPU restatement of "
                      "OPA v0.21 topdown; Go/OPA not buildable offline" % (len(reviews), len(constraints)),
            "latency_ms_per_request": {"p50": lat[len(lat) // 2], "p99": lat[min(len(lat) - 1, int(0.99 * len(lat)))]},
            "batch_latency_ms": tot * 1000.0, "seconds": tot}


if __name__ == "__main__":
    main()
