"""ORACLE fixture generator (test infrastructure only; container-side).

Runs the REFERENCE code from /root/reference (read-only) and freezes its outputs
as small fixtures under tests/golden/, plus a minimal topology .inp (only the
sections the graph builder reads) under leak-det-gnn_amd/data/ so the GPU box,
which has no /root/reference, can construct the L-TOWN-A detector.

  python oracle/make_golden.py [--ref /root/reference]

Reference modules imported as-is: models/utils.py, models/predictor.py.
models/detector.py imports torch_geometric (absent, unpinned); it is run with
the independent dense formulation oracle/dense_ref.py supplied as
torch_geometric.nn, so every non-PyG step of the fixture is the reference's own
code and the PyG steps are the dense restatement (recorded in meta).
"""
from __future__ import annotations

import argparse
import json
import sys
import types
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
GOLD = REPO / "tests" / "golden"
DATA = REPO / "leak-det-gnn_amd" / "data"
SENSORS = ['n54', 'n105', 'n114', 'n163', 'n188', 'n229', 'n288', 'n296', 'n332', 'n342', 'n410', 'n415', 'n429',
           'n458', 'n469', 'n495', 'n506', 'n516', 'n519', 'n549', 'n613', 'n636', 'n644', 'n679', 'n722', 'n726',
           'n740', 'n752', 'n769']  # configs/sim_LTA.yaml:21


def _import_reference(ref: Path):
    sys.path.insert(0, str(REPO))
    from oracle import dense_ref  # noqa: E402
    tg = types.ModuleType("torch_geometric")
    tgnn = types.ModuleType("torch_geometric.nn")
    tgnn.GCNConv = dense_ref.GCNConv
    tgnn.global_mean_pool = dense_ref.global_mean_pool
    tg.nn = tgnn
    sys.modules["torch_geometric"] = tg
    sys.modules["torch_geometric.nn"] = tgnn
    sys.path.insert(0, str(ref))
    import models.utils as rutils  # noqa: E402
    import models.predictor as rpred  # noqa: E402
    import models.detector as rdet  # noqa: E402
    return rutils, rpred, rdet


def write_topology_inp(rutils, src: Path, dst: Path) -> None:
    sec = rutils.parse_epanet_inp(src)
    keep = ["JUNCTIONS", "RESERVOIRS", "TANKS", "PIPES", "PUMPS", "VALVES"]
    lines = [f"[TITLE]", f"topology extracted from {src.name} by oracle/make_golden.py (ids, link endpoints and "
             f"pipe lengths only)", ""]
    for s in keep:
        lines.append(f"[{s}]")
        for ln in sec.get(s, []):
            tok = ln.split()
            # pipes keep their length (distance metrics, window_evaluator.py:76-110)
            lines.append(" ".join(tok[:4]) if s == "PIPES" else " ".join(tok[:3]) if s in ("PUMPS", "VALVES")
                         else tok[0])
        lines.append("")
    lines.append("[END]")
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text("\n".join(lines) + "\n", encoding="utf-8")


def graph_fixture(rutils, rdet, inp: Path, sensors, out: Path) -> dict:
    sec = rutils.parse_epanet_inp(inp)
    pipe_ids = sorted(rutils._parse_links(sec["PIPES"]).keys())  # all pipes, dataset order (datasets.py:353)
    node_set = set()
    for s in ("JUNCTIONS", "RESERVOIRS", "TANKS"):
        node_set.update(rutils._parse_nodes(sec.get(s, [])))
    sensors = [s for s in sensors if s in node_set]
    g = rutils.build_wdn_graph_from_inp(inp, sensors, pipe_ids, add_self_loops=False, make_undirected=True)
    ei = g.edge_index
    bat = rdet._batchify_edge_index(ei, len(g.node_names), 3)
    g2 = rutils.build_wdn_graph_from_inp(inp, sensors, pipe_ids, add_self_loops=True, make_undirected=False)
    np.savez_compressed(out, node_names=np.array(g.node_names), pipe_ids=np.array(pipe_ids),
                        sensor_ids=np.array(sensors), edge_index=ei.numpy(), pipe_ends=g.pipe_ends,
                        sensor_node_idx=np.array([g.node_to_idx[s] for s in sensors], dtype=np.int64),
                        batchified_b3=bat.numpy(), edge_index_loops_directed=g2.edge_index.numpy())
    return {"nodes": len(g.node_names), "edges": int(ei.shape[1]), "pipes": len(pipe_ids)}


def detector_fixture(rdet, inp: Path, pipe_ids, B: int, out: Path, with_state: bool, with_trace: bool) -> None:
    torch.manual_seed(0)
    model = rdet.LeakDetector(inp, SENSORS, pipe_ids, sensor_hidden=64, node_hidden=64, gnn_layers=2, dropout=0.1,
                              use_time=True)
    model.eval()
    trace = {}
    hooks = [model.sensor_to_node.register_forward_hook(lambda m, i, o: trace.__setitem__("node_init", torch.relu(o)))]
    for k, conv in enumerate(model.convs):
        hooks.append(conv.register_forward_hook(lambda m, i, o, k=k: trace.__setitem__(f"conv{k}", torch.relu(o))))
    g = torch.Generator().manual_seed(1000 + B)
    residual = torch.randn(B, 36, len(SENSORS), generator=g).requires_grad_(True)
    tfeat = torch.randn(B, 36, 9, generator=g)
    label = torch.randint(0, len(pipe_ids) + 1, (B,), generator=g)
    logits = model(residual, tfeat)
    loss = torch.nn.functional.cross_entropy(logits, label)
    loss.backward()
    for h in hooks:
        h.remove()
    arrs = dict(residual=residual.detach().numpy(), tfeat=tfeat.numpy(), label=label.numpy(),
                logits=logits.detach().numpy(), loss=np.array(loss.item(), dtype=np.float32),
                grad_residual=residual.grad.numpy())
    for name, p in model.named_parameters():
        arrs["grad." + name] = p.grad.numpy()
        if with_state:
            arrs["param." + name] = p.detach().numpy()
    if with_trace:
        for k, v in trace.items():
            arrs["trace." + k] = v.detach().reshape(B, -1, v.shape[-1]).numpy()
    np.savez_compressed(out, **arrs)


def predictor_fixture(rutils, rpred, out: Path) -> None:
    torch.manual_seed(0)
    tcn = rpred.NormalPredictorTCN(num_sensors=29, time_dim=9).eval()
    torch.manual_seed(0)
    gru = rpred.NormalPredictorGRU(num_sensors=29, time_dim=9).eval()
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 36, 29, generator=g)
    xt = torch.randn(4, 36, 9, generator=g)
    seg = torch.randn(2, 72, 29, generator=g)
    tseg = torch.randn(2, 72, 9, generator=g)
    with torch.no_grad():
        y_tcn = tcn(x, xt)
        y_gru = gru(x, xt)
        res = rutils.build_residual_sequence_from_segment(tcn, seg, tseg, l_pred=36, l_det=36)
    arrs = dict(x=x.numpy(), x_time=xt.numpy(), y_tcn=y_tcn.numpy(), y_gru=y_gru.numpy(), seg=seg.numpy(),
                tseg=tseg.numpy(), residual=res.numpy())
    for n, p in tcn.state_dict().items():
        arrs["tcn." + n] = p.numpy()
    for n, p in gru.state_dict().items():
        arrs["gru." + n] = p.numpy()
    np.savez_compressed(out, **arrs)


class FixedLogitsDetector(torch.nn.Module):
    """Deterministic stand-in detector for the evaluator fixture (weights stored in the
    fixture): logits = 3 tanh(mean_t(residual) A + mean_t(tfeat) Bm) + c."""

    def __init__(self, A, Bm, c):
        super().__init__()
        self.A, self.Bm, self.c = (torch.as_tensor(v, dtype=torch.float32) for v in (A, Bm, c))

    def forward(self, residual, tfeat):
        dev = residual.device
        return 3.0 * torch.tanh(residual.mean(1) @ self.A.to(dev) + tfeat.mean(1) @ self.Bm.to(dev)) + self.c.to(dev)


def harness_fixture(ref: Path, rpred, lta_inp: Path, pipe_pool, out_npz: Path, out_json: Path) -> dict:
    """Data-pipeline / trainer-split / evaluator fixtures: the reference's own
    models/datasets.py, train_detector.py split functions and window_evaluator.py run on
    a seeded synthetic data set written by models/synth.py (regenerated by the tests)."""
    import importlib.util
    import tempfile
    # the product's data writer, loaded standalone (both code bases name their package `models`)
    spec = importlib.util.spec_from_file_location("lg_synth", REPO / "leak-det-gnn_amd" / "models" / "synth.py")
    lg_synth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lg_synth)
    write_synthetic_leak_set, write_synthetic_normal_set = lg_synth.write_synthetic_leak_set, \
        lg_synth.write_synthetic_normal_set
    import models.datasets as rds  # the reference's
    import models.train_detector as rtd
    import models.window_evaluator as rwe
    assert str(ref) in rds.__file__, rds.__file__
    pipes = [pipe_pool[i] for i in (3, 50, 120, 333, 500, 700)]
    arrs, info = {}, {"pipes": pipes, "sensors": SENSORS}
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        write_synthetic_normal_set(d / "normal", SENSORS, n_windows=12, T=577, seed=0)
        write_synthetic_leak_set(d / "leak", SENSORS, pipes, scenes_per_pipe=2, n_noleak=6, T=400, seed=0)
        st = rds.compute_sensor_stats_from_normal(d / "normal")
        arrs["std_mean"], arrs["std_std"] = st.mean, st.std
        nds = rds.NormalPredictorDataset(d / "normal", steps_per_epoch=50, seed=42, standardizer=st)
        info["normal_samples"] = []
        for i in range(8):
            smp = nds[i]
            info["normal_samples"].append({"scene_id": str(smp["scene_id"]), "t": smp["t"]})
            for k in ("x", "x_time", "y"):
                arrs[f"normal.{i}.{k}"] = smp[k].numpy()
        lds = rds.AbruptLeakDetectorDataset(d / "leak", steps_per_epoch=64, seed=123, standardizer=st,
                                            sensor_ids=SENSORS)
        info["leak_scene_ids"] = [str(x) for x in lds.leak_scene_ids]
        info["noleak_scene_ids"] = [str(x) for x in lds.noleak_scene_ids]
        info["pipe_ids_in_order"] = lds.get_pipe_ids_in_order()
        info["bucket_sizes"] = {sid: {b: int(v.size) for b, v in bt.items()} for sid, bt in lds._bucket_times.items()}
        info["leak_samples"] = []
        for i in range(24):
            smp = lds[i]
            info["leak_samples"].append({k: (str(v) if k in ("scenario_id", "bucket", "t", "pipe_id") else int(v))
                                         for k, v in smp.items() if k not in ("noisy_seg", "time_seg")})
            arrs[f"leak.{i}.noisy_seg"] = smp["noisy_seg"].numpy()
            arrs[f"leak.{i}.time_seg"] = smp["time_seg"].numpy()
        # trainer splits on a larger id list
        fake = [f"{k:06d}_p{k % 12}_abrupt_r{k // 12 + 1}" for k in range(50)]
        info["split_leak"] = [list(x) for x in rtd.split_leak_scenids(fake, 42, ratio=(0.8, 0.1, 0.1))]
        info["split_normal"] = [list(x) for x in rtd.split_normal_scenids([f"w{k}" for k in range(23)], 53)]
        # evaluator on a fixed predictor + stand-in detector
        torch.manual_seed(0)
        tcn = rpred.NormalPredictorTCN(num_sensors=29, time_dim=9).eval()
        g = torch.Generator().manual_seed(11)
        P1 = len(pipes) + 1
        A, Bm, c = torch.randn(29, P1, generator=g), torch.randn(9, P1, generator=g), torch.randn(P1, generator=g)
        arrs["eval.A"], arrs["eval.Bm"], arrs["eval.c"] = A.numpy(), Bm.numpy(), c.numpy()
        det = FixedLogitsDetector(A, Bm, c)
        eds = rds.AbruptLeakDetectorDataset(d / "leak", steps_per_epoch=48, seed=7, standardizer=st,
                                            sensor_ids=SENSORS)
        ev = rwe.DetectorEvaluator(tcn, det, torch.device("cpu"), l_pred=36, l_det=36, topk=5,
                                   metric_groups=("basic", "binary", "bucket", "atd", "success", "accuracy_i"),
                                   inp_path=lta_inp, pipe_ids_in_order=lds.get_pipe_ids_in_order())
        from torch.utils.data import DataLoader
        info["eval_metrics"] = {k: float(v) for k, v in ev.evaluate(DataLoader(eds, batch_size=16)).items()}
    np.savez_compressed(out_npz, **arrs)
    out_json.write_text(json.dumps(info, indent=1) + "\n")
    return {"normal_samples": 8, "leak_samples": 24, "eval_metrics": len(info["eval_metrics"])}


NOLEAK_BIAS = (2.0, 3.0)


def event_fixture(ref: Path, lta_inp: Path, out_json: Path) -> dict:
    """Event-level evaluator fixture: the reference's eval/event_evaluator.py
    (`evaluate_dataset_event_level`, B = 1 per stride step) on the synthetic leak set,
    the seeded TCN of predictor.npz and the stand-in detector of harness.npz; records
    the per-event jsonl and summary.json it writes."""
    import importlib.util
    import tempfile
    spec = importlib.util.spec_from_file_location("lg_synth", REPO / "leak-det-gnn_amd" / "models" / "synth.py")
    lg_synth = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lg_synth)
    spec = importlib.util.spec_from_file_location("ref_event_evaluator", ref / "eval" / "event_evaluator.py")
    rev = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(rev)
    import models.predictor as rpred  # the reference's (path set by _import_reference)
    info = json.loads((GOLD / "harness.json").read_text())
    h = np.load(GOLD / "harness.npz")
    p = np.load(GOLD / "predictor.npz")
    tcn = rpred.NormalPredictorTCN(num_sensors=29, time_dim=9).eval()
    tcn.load_state_dict({k[4:]: torch.from_numpy(p[k]) for k in p.files if k.startswith("tcn.")})
    std = rev.SensorStandardizer(mean=h["std_mean"], std=h["std_std"])
    # noleak_bias lifts the stand-in's no-leak logit so alarms come late, or never
    cases = [dict(stride_steps=3, agg_window_hours=1.0, include_noleak=True, max_leak_scens=8, max_noleak_scens=4),
             dict(stride_steps=1, agg_window_hours=12.0, include_noleak=True, max_leak_scens=-1, max_noleak_scens=-1),
             dict(stride_steps=2, agg_window_hours=2.0, include_noleak=True, max_leak_scens=-1, max_noleak_scens=-1,
                  noleak_bias=NOLEAK_BIAS[0]),
             dict(stride_steps=1, agg_window_hours=0.5, include_noleak=False, max_leak_scens=5, max_noleak_scens=2,
                  noleak_bias=NOLEAK_BIAS[1])]
    out = {"pipes": info["pipes"], "l_pred": 36, "l_det": 36, "cases": []}
    with tempfile.TemporaryDirectory() as d:
        d = Path(d)
        lg_synth.write_synthetic_leak_set(d / "leak", SENSORS, info["pipes"], scenes_per_pipe=2, n_noleak=6, T=400,
                                          seed=0)
        for c in cases:
            kw = {k: v for k, v in c.items() if k != "noleak_bias"}
            cc = h["eval.c"].copy()
            cc[-1] += np.float32(c.get("noleak_bias", 0.0))
            det = FixedLogitsDetector(h["eval.A"], h["eval.Bm"], cc)
            summary = rev.evaluate_dataset_event_level(
                d / "leak", lta_inp, torch.device("cpu"), tcn, det, 36, 36, std, SENSORS, info["pipes"],
                sample_seed=42, out_dir=d / "out", **kw)
            events = [json.loads(ln) for ln in (d / "out" / "per_event.jsonl").read_text().splitlines() if ln]
            out["cases"].append({"args": c, "summary": summary, "events": events})
    out_json.write_text(json.dumps(out, indent=1) + "\n")
    return {"cases": len(cases), "events": [len(c["events"]) for c in out["cases"]]}


RESIDUAL_CASES = ((36, 36, 3), (12, 20, 2), (64, 8, 2), (40, 1, 2))  # (l_pred, l_det, B)


def residual_fixture(rutils, rpred, out: Path) -> dict:
    """Residual builder (utils.py:169-216) on a TCN with non-trivial LayerNorm affine and
    conv biases, at several (l_pred, l_det): pins the shared-window row plan beyond the
    default 36/36 case."""
    torch.manual_seed(3)
    tcn = rpred.NormalPredictorTCN(num_sensors=29, time_dim=9).eval()
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for blk in tcn.tcn:
            for norm in (blk.norm1, blk.norm2):
                norm.weight.copy_(1.0 + 0.5 * torch.randn(norm.weight.shape, generator=g))
                norm.bias.copy_(0.3 * torch.randn(norm.bias.shape, generator=g))
    arrs = {"tcn." + n: p.numpy() for n, p in tcn.state_dict().items()}
    arrs["cases"] = np.array(RESIDUAL_CASES, dtype=np.int64)
    for i, (lp, ld, B) in enumerate(RESIDUAL_CASES):
        seg = torch.randn(B, lp + ld, 29, generator=g)
        tseg = torch.randn(B, lp + ld, 9, generator=g)
        with torch.no_grad():
            res = rutils.build_residual_sequence_from_segment(tcn, seg, tseg, l_pred=lp, l_det=ld)
        arrs[f"seg{i}"], arrs[f"tseg{i}"], arrs[f"res{i}"] = seg.numpy(), tseg.numpy(), res.numpy()
    np.savez_compressed(out, **arrs)
    return {"cases": [list(c) for c in RESIDUAL_CASES]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", choices=["residual", "event"], default=None,
                    help="regenerate one fixture only (leaves the others byte-identical)")
    args = ap.parse_args()
    ref = Path(args.ref)
    rutils, rpred, rdet = _import_reference(ref)
    GOLD.mkdir(parents=True, exist_ok=True)
    if args.only == "event":
        meta = json.loads((GOLD / "meta.json").read_text())
        meta["event"] = event_fixture(ref, ref / "data/raw/L-TOWN-A/L-TOWN_AreaA.inp", GOLD / "event.json")
        (GOLD / "meta.json").write_text(json.dumps(meta, indent=2) + "\n")
        return
    if args.only == "residual":
        meta = json.loads((GOLD / "meta.json").read_text())
        meta["residual"] = residual_fixture(rutils, rpred, GOLD / "residual.npz")
        (GOLD / "meta.json").write_text(json.dumps(meta, indent=2) + "\n")
        return
    lta = ref / "data/raw/L-TOWN-A/L-TOWN_AreaA.inp"
    lt = ref / "data/raw/L-TOWN/L-TOWN.inp"
    write_topology_inp(rutils, lta, DATA / "L-TOWN-A.inp")
    meta = {"generator": "oracle/make_golden.py", "reference": str(ref),
            "pyg": "absent/unpinned; detector fixtures use oracle/dense_ref.py as torch_geometric.nn",
            "torch": torch.__version__}
    meta["graph_ltown_a"] = graph_fixture(rutils, rdet, lta, SENSORS, GOLD / "graph_ltown_a.npz")
    meta["graph_ltown"] = graph_fixture(rutils, rdet, lt, SENSORS, GOLD / "graph_ltown.npz")
    pipe_ids = [str(p) for p in np.load(GOLD / "graph_ltown_a.npz")["pipe_ids"]]
    detector_fixture(rdet, lta, pipe_ids, 2, GOLD / "detector_b2.npz", with_state=True, with_trace=True)
    detector_fixture(rdet, lta, pipe_ids, 8, GOLD / "detector_b8.npz", with_state=False, with_trace=False)
    predictor_fixture(rutils, rpred, GOLD / "predictor.npz")
    meta["residual"] = residual_fixture(rutils, rpred, GOLD / "residual.npz")
    meta["harness"] = harness_fixture(ref, rpred, lta, pipe_ids, GOLD / "harness.npz", GOLD / "harness.json")
    meta["event"] = event_fixture(ref, lta, GOLD / "event.json")
    (GOLD / "meta.json").write_text(json.dumps(meta, indent=2) + "\n")
    print(json.dumps(meta, indent=2))


if __name__ == "__main__":
    main()
