"""Generate the golden fixtures under tests/golden/ (run HERE, where /root/reference exists).

    python tests/golden/make_golden.py

What it does (nothing here ships or runs on the GPU box):
  * AST-loads ONLY the ClassDef/FunctionDef nodes of the reference model/loss code from
    /root/reference/src/{Convolutional_VAE,Conditional_VAE,Simple_VAE}.py (their module top
    levels load data from hard-coded Windows paths, so they cannot be imported whole — SURVEY §8c).
    For 128x128 inputs the flatten literals (16384, (512, 2, 16)) are rewritten in the AST to
    F = 512*(H/64)*(W/64); at 128x1024 nothing is rewritten.
  * Runs the reference classes on CPU from torch.manual_seed(42) init with seeded inputs and
    host-supplied eps (torch.randn_like is patched for the reference's reparameterize), and records
    outputs, losses, gradient summaries and 1- / 3-step Adam states.
  * Checks that oracle/models_oracle.py (the restatement used on the GPU box) reproduces every
    recorded value bit-for-bit, and fails otherwise.
  * Records sklearn 1.7.2 KMeans(random_state=42, n_init=10) labels on seeded blob data, the sklearn.metrics
    scores of those labels (silhouette incl. per-sample, Davies-Bouldin, Calinski-Harabasz, ARI, NMI) and the
    reference's own calculate_purity, and the oracle's mel / MFCC / pooling outputs on seeded synthetic PCM.
Fixtures are data (inputs + expected outputs); no reference source is stored.
"""
from __future__ import annotations

import ast
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
REF = "/root/reference/src"

from oracle import mel_oracle, models_oracle  # noqa: E402
from tests.golden import fixtures  # noqa: E402


class _FlattenRewrite(ast.NodeTransformer):
    def __init__(self, flat, unflat):
        self.flat, self.unflat = flat, unflat

    def visit_Constant(self, node):
        if node.value == 16384 and self.flat != 16384:
            return ast.copy_location(ast.Constant(self.flat), node)
        return node

    def visit_Tuple(self, node):
        self.generic_visit(node)
        vals = [getattr(e, "value", None) for e in node.elts]
        if vals == [512, 2, 16]:
            return ast.copy_location(ast.Tuple([ast.Constant(v) for v in self.unflat], ast.Load()), node)
        return node


class _AudioOnlyRewrite(ast.NodeTransformer):
    """BASELINE config[1]'s audio-only ConvVAE from the reference HybridVAE / loss_function:
    the text branch, its fusion slice and its loss term removed, everything else untouched.

      * ``self.text_encoder = ...`` / ``self.text_decoder = ...`` registrations dropped (src/Convolutional_VAE.py
        :103-110, :142-147), so the remaining modules draw the same torch.manual_seed stream as the restatement;
      * ``t = self.text_encoder(text)`` dropped and ``torch.cat((a, t), dim=1)`` -> ``a`` (:153-155);
      * the fusion slice ``1024 + 128`` -> ``1024`` in fc_fusion and decoder_split (:112, :118);
      * ``recon_text = self.text_decoder(t_hidden)`` -> ``None`` (:177);
      * loss: ``recon_loss_text`` -> a zero scalar and the ``recon_loss_text * 350`` term removed (:190, :194).
    Every rewrite is counted; a reference that no longer has exactly these sites fails loudly."""

    EXPECT = {"drop_module": 2, "drop_text_call": 1, "cat": 1, "slice": 2, "recon_text": 1, "loss_text": 1,
              "loss_term": 1}

    def __init__(self):
        self.n = {k: 0 for k in self.EXPECT}
        self.dropped = set()

    @staticmethod
    def _is_self_attr(node, names):
        return (isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name) and node.value.id == "self"
                and node.attr in names)

    def _calls(self, node, attr):
        return isinstance(node, ast.Call) and self._is_self_attr(node.func, {attr})

    def visit_Assign(self, node):
        tgt = node.targets[0]
        if self._is_self_attr(tgt, {"text_encoder", "text_decoder"}):
            self.n["drop_module"] += 1
            return None
        if self._calls(node.value, "text_encoder"):
            self.n["drop_text_call"] += 1
            self.dropped.add(tgt.id)
            return None
        if self._calls(node.value, "text_decoder"):
            self.n["recon_text"] += 1
            node.value = ast.Constant(None)
            return node
        if (isinstance(tgt, ast.Name) and tgt.id == "recon_loss_text" and isinstance(node.value, ast.Call)
                and getattr(node.value.func, "attr", None) == "mse_loss"):
            self.n["loss_text"] += 1
            node.value = ast.parse("torch.zeros_like(recon_loss_audio)", mode="eval").body
            return node
        self.generic_visit(node)
        return node

    def visit_Call(self, node):
        self.generic_visit(node)
        if (isinstance(node.func, ast.Attribute) and node.func.attr == "cat" and node.args
                and isinstance(node.args[0], ast.Tuple)):
            elts = [e for e in node.args[0].elts if not (isinstance(e, ast.Name) and e.id in self.dropped)]
            if len(elts) == 1 and len(node.args[0].elts) == 2:
                self.n["cat"] += 1
                return elts[0]
        return node

    def visit_BinOp(self, node):
        self.generic_visit(node)
        if (isinstance(node.op, ast.Add) and isinstance(node.left, ast.Constant) and isinstance(node.right, ast.Constant)
                and (node.left.value, node.right.value) == (1024, 128)):
            self.n["slice"] += 1
            return ast.copy_location(ast.Constant(1024), node)
        r = node.right
        if (isinstance(node.op, ast.Add) and isinstance(r, ast.BinOp) and isinstance(r.op, ast.Mult)
                and isinstance(r.left, ast.Name) and r.left.id == "recon_loss_text"):
            self.n["loss_term"] += 1
            return node.left
        return node

    def check(self):
        if self.n != self.EXPECT:
            raise AssertionError(f"audio-only rewrite sites differ from the reference: {self.n} != {self.EXPECT}")


def load_reference(fname, names, input_hw=(128, 1024), audio_only=False):
    src = open(os.path.join(REF, fname)).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef)) and n.name in names]
    flat, unflat = models_oracle.flat_dims(input_hw)
    mod = ast.Module(body=keep, type_ignores=[])
    mod = _FlattenRewrite(flat, unflat).visit(mod)
    if audio_only:
        rw = _AudioOnlyRewrite()
        mod = rw.visit(mod)
        rw.check()
    mod = ast.fix_missing_locations(mod)
    ns = {"torch": torch, "nn": nn, "np": np}
    exec(compile(mod, f"<reference {fname}>", "exec"), ns)
    return ns


class _EpsPatch:
    """Make torch.randn_like return host-supplied eps inside the reference's reparameterize."""

    def __init__(self, eps):
        self.eps = eps

    def __enter__(self):
        self.orig = torch.randn_like
        torch.randn_like = lambda t, *a, **k: self.eps.clone()

    def __exit__(self, *exc):
        torch.randn_like = self.orig


def _assert_same(a, b, what):
    if isinstance(a, torch.Tensor):
        if not torch.equal(a, b):
            raise AssertionError(f"restatement != reference for {what}: max|d|={(a - b).abs().max().item()}")


def run_case(kind, ref_cls, ref_loss, ora_cls, ora_loss, ctor, ora_ctor, inputs_fn, loss_kw, steps=3):
    """Run reference & restatement side by side; return a dict of fixture arrays."""
    out = {}
    torch.manual_seed(42)
    ref = ref_cls(**ctor)
    torch.manual_seed(42)
    ora = ora_cls(**ora_ctor)
    sr, so = ref.state_dict(), ora.state_dict()
    assert list(sr.keys()) == list(so.keys()), f"{kind}: state_dict keys differ"
    for k in sr:
        _assert_same(sr[k], so[k], f"{kind} init {k}")
    names = [n for n, _ in ref.named_parameters()]
    out["param_names"] = np.array(names)
    out["param_checksum_init"] = fixtures.param_summary(ref)
    opt_r = torch.optim.Adam(ref.parameters(), lr=1e-4)
    opt_o = torch.optim.Adam(ora.parameters(), lr=1e-4)
    for step in range(steps):
        ins, eps = inputs_fn(step)
        for m in (ref, ora):
            m.train()
        opt_r.zero_grad()
        opt_o.zero_grad()
        torch.manual_seed(7 + step)          # identical dropout masks (Simple VAE) for both
        with _EpsPatch(eps):
            ro = ref(*ins)
        torch.manual_seed(7 + step)
        oo = ora(*ins, eps=eps)
        lr_ = ref_loss(*fixtures.loss_args(kind, ro, ins), **loss_kw)
        lo_ = ora_loss(*fixtures.loss_args(kind, oo, ins), **loss_kw)
        for i, (a, b) in enumerate(zip(ro, oo)):
            _assert_same(a, b, f"{kind} step{step} output{i}")
        for i, (a, b) in enumerate(zip(lr_, lo_)):
            _assert_same(a, b, f"{kind} step{step} loss{i}")
        lr_[0].backward()
        lo_[0].backward()
        for (n, p), q in zip(ref.named_parameters(), ora.parameters()):
            _assert_same(p.grad, q.grad, f"{kind} step{step} grad {n}")
        if step == 0:
            for i, t in enumerate(ro):
                if isinstance(t, torch.Tensor):
                    out[f"out{i}"] = t.detach().numpy()
            out["grad_summary"] = fixtures.grad_summary(ref)
        out[f"loss_step{step}"] = np.array([float(t) for t in lr_], dtype=np.float64)
        opt_r.step()
        opt_o.step()
        if step in (0, steps - 1):
            out[f"param_summary_after{step + 1}"] = fixtures.param_summary(ref)
            out[f"buffer_summary_after{step + 1}"] = fixtures.buffer_summary(ref)
    for m in (ref, ora):
        m.eval()
    ins, _ = inputs_fn(0)
    with torch.no_grad():
        mu_r = ref.encode(*fixtures.encode_args(kind, ins))[0]
        mu_o = ora.encode(*fixtures.encode_args(kind, ins))[0]
    _assert_same(mu_r, mu_o, f"{kind} eval mu")
    out["eval_mu"] = mu_r.numpy()
    return out


def make_models(only=None):
    conv = lambda hw, ao=False: load_reference("Convolutional_VAE.py", {"HybridVAE", "loss_function"}, hw, ao)  # noqa: E731
    cond = lambda hw: load_reference("Conditional_VAE.py", {"ConditionalVAE", "cvae_loss_function", "SimpleAutoencoder"}, hw)  # noqa: E731
    simple = load_reference("Simple_VAE.py", {"VAE", "vae_loss"})
    for case in fixtures.MODEL_CASES:
        kind, hw = case["kind"], case.get("hw")
        if only and case["name"] not in only:
            continue
        print("case", case["name"], flush=True)
        if kind == "hybrid":
            ns = conv(hw, bool(case.get("audio_only")))
            res = run_case(kind, ns["HybridVAE"], ns["loss_function"], models_oracle.HybridVAE,
                           models_oracle.loss_function, case["ctor"], fixtures.oracle_ctor(case), fixtures.inputs_fn(case), {})
        elif kind == "cvae":
            ns = cond(hw)
            res = run_case(kind, ns["ConditionalVAE"], ns["cvae_loss_function"], models_oracle.ConditionalVAE,
                           models_oracle.cvae_loss_function, case["ctor"], fixtures.oracle_ctor(case), fixtures.inputs_fn(case), {"beta": 4.0})
        elif kind == "simple":
            res = run_case(kind, simple["VAE"], simple["vae_loss"], models_oracle.VAE, models_oracle.vae_loss,
                           case["ctor"], fixtures.oracle_ctor(case), fixtures.inputs_fn(case), {"beta": 0.8})
        else:
            raise ValueError(kind)
        np.savez_compressed(os.path.join(HERE, f"model_{case['name']}.npz"), **res)
    if only:
        return
    # SimpleAutoencoder: forward only (the CVAE baseline)
    ns = cond((128, 1024))
    torch.manual_seed(42)
    ae_r = ns["SimpleAutoencoder"](290, 64)
    torch.manual_seed(42)
    ae_o = models_oracle.SimpleAutoencoder(290, 64)
    x = torch.randn(8, 290, generator=torch.Generator().manual_seed(3))
    for a, b in zip(ae_r(x), ae_o(x)):
        _assert_same(a, b, "SimpleAutoencoder")
    print("restatement == reference (bit-exact) for all model cases", flush=True)


def make_kmeans():
    from sklearn.cluster import KMeans
    from threadpoolctl import threadpool_limits
    for (n, d, centers, k, n_init) in fixtures.KMEANS_CASES:
        X = fixtures.blobs(n, d, centers, seed=n + d + k)
        with threadpool_limits(1):
            km = KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)
        np.savez_compressed(os.path.join(HERE, f"kmeans_n{n}_d{d}_k{k}_i{n_init}.npz"),
                            labels=km.labels_.astype(np.int16), centers=km.cluster_centers_.astype(np.float32),
                            inertia=np.float64(km.inertia_), n_iter=np.int32(km.n_iter_))
        print("kmeans", n, d, k, n_init, km.n_iter_, flush=True)


def _sk_kmeans(X, k, n_init):
    from sklearn.cluster import KMeans
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):   # one OpenMP thread: sklearn's row-order centre sums are deterministic
        return KMeans(n_clusters=k, random_state=42, n_init=n_init).fit(X)


def make_kmeans_overlap():
    """Overlapping clusters (near-tie E-steps) and the config[4]-scale case (N = 100 000)."""
    for case in fixtures.KMEANS_OVERLAP_CASES + [fixtures.KMEANS_BIG_CASE]:
        n, d, true_k, spread, k, n_init = case
        X = fixtures.overlap_blobs(n, d, true_k, spread, fixtures.overlap_seed(case))
        km = _sk_kmeans(X, k, n_init)
        np.savez_compressed(os.path.join(HERE, fixtures.overlap_fixture_name(case)),
                            labels=km.labels_.astype(np.int16), centers=km.cluster_centers_.astype(np.float32),
                            inertia=np.float64(km.inertia_), n_iter=np.int32(km.n_iter_))
        print("kmeans overlap", case, km.n_iter_, flush=True)


def latent_dataset():
    """Eval-mode mu of the oracle HybridVAE (128x128, text 768) on LATENT_N synthetic clips: oracle mel-dB ->
    per-pixel z-score -> 5 train-mode Adam steps (so BatchNorm running statistics are real) -> eval encode."""
    import torch
    n = fixtures.LATENT_N
    pcm = mel_oracle.synthetic_pcm(n, 65024, seed=2024)
    mel = np.stack([mel_oracle.extract_mel_spectrogram(c) for c in pcm]).astype(np.float32)
    z = ((mel - mel.mean(0)) / (mel.std(0) + 1e-8)).astype(np.float32)
    g = torch.Generator().manual_seed(5)
    text = torch.randn(n, 768, generator=g) / 768 ** 0.5
    audio = torch.from_numpy(z)[:, None]
    torch.manual_seed(42)
    model = models_oracle.HybridVAE(128, 768, (128, 128))
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    model.train()
    for step in range(5):
        idx = torch.arange(step * 32, step * 32 + 32)
        eps = torch.randn(32, 128, generator=g)
        out = model(audio[idx], text[idx], eps=eps)
        loss = models_oracle.loss_function(out[0], audio[idx], out[1], text[idx], out[2], out[3])[0]
        opt.zero_grad()
        loss.backward()
        opt.step()
    model.eval()
    with torch.no_grad():
        mu = torch.cat([model.encode(audio[i:i + 128], text[i:i + 128])[0] for i in range(0, n, 128)])
    return mu.numpy().astype(np.float32)


def make_kmeans_latents():
    X = latent_dataset()
    out = {"X": X}
    for k in fixtures.LATENT_KS:
        km = _sk_kmeans(X, k, 10)
        out[f"labels_k{k}"] = km.labels_.astype(np.int16)
        out[f"centers_k{k}"] = km.cluster_centers_.astype(np.float32)
        out[f"inertia_k{k}"] = np.float64(km.inertia_)
        out[f"n_iter_k{k}"] = np.int32(km.n_iter_)
        print("kmeans latents k", k, km.n_iter_, flush=True)
    np.savez_compressed(os.path.join(HERE, "kmeans_latents_n1336_d128.npz"), **out)


def make_metrics():
    """sklearn.metrics scores of the K-Means fixture labels (and the blob ground truth), plus the reference's own
    calculate_purity (src/Conditional_VAE.py:279-287, AST-loaded) — §8f rows 1 and 4."""
    from sklearn import metrics as skm
    src = open(os.path.join(REF, "Conditional_VAE.py")).read()
    tree = ast.parse(src)
    keep = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "calculate_purity"]
    ns = {"np": np, "confusion_matrix": skm.confusion_matrix}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "Conditional_VAE.py", "exec"), ns)
    purity = ns["calculate_purity"]
    for case in fixtures.METRICS_CASES:
        n, d, centers, k, n_init = case
        X = fixtures.blobs(n, d, centers, seed=n + d + k)
        y_true = fixtures.blob_labels(n, d, centers, seed=n + d + k)
        y_pred = np.load(os.path.join(HERE, fixtures.kmeans_fixture_name(case)))["labels"].astype(np.int64)
        np.savez_compressed(os.path.join(HERE, fixtures.metrics_fixture_name(case)),
                            silhouette=np.float64(skm.silhouette_score(X, y_pred)),
                            silhouette_samples=skm.silhouette_samples(X, y_pred).astype(np.float64),
                            davies_bouldin=np.float64(skm.davies_bouldin_score(X, y_pred)),
                            calinski_harabasz=np.float64(skm.calinski_harabasz_score(X, y_pred)),
                            ari=np.float64(skm.adjusted_rand_score(y_true, y_pred)),
                            nmi=np.float64(skm.normalized_mutual_info_score(y_true, y_pred)),
                            purity=np.float64(purity(y_true, y_pred)))
        print("metrics", n, d, k, flush=True)


def make_features():
    from sklearn.preprocessing import StandardScaler
    y = mel_oracle.synthetic_pcm(2, 65024, seed=7)
    mel = np.stack([mel_oracle.extract_mel_spectrogram(c) for c in y])
    mf = np.stack([mel_oracle.mfcc(c) for c in y])
    pool = np.stack([np.concatenate([mel_oracle.mean_std_pool(a), mel_oracle.mean_std_pool(b)]) for a, b in zip(mel, mf)])
    rng = np.random.default_rng(11)
    cols = (rng.standard_normal((64, 300)) * rng.uniform(0.1, 5, 300) + rng.uniform(-3, 3, 300)).astype(np.float32)
    cols[:, 5] = 2.5
    sc = StandardScaler().fit(cols)
    np.savez_compressed(os.path.join(HERE, "features.npz"), mel_db=mel, mfcc=mf, pool=pool,
                        mel_basis=mel_oracle.mel_filterbank(), scaler_mean=sc.mean_,
                        scaler_var=sc.var_, scaler_scale=sc.scale_, scaler_out=sc.transform(cols))
    print("features done", flush=True)


if __name__ == "__main__":
    torch.set_num_threads(8)
    what = sys.argv[1:] or ["models", "kmeans", "kmeans_overlap", "kmeans_latents", "metrics", "features"]
    # "models=<case>[,<case>]" regenerates only the named model fixtures
    only = [c for w in what if w.startswith("models=") for c in w.split("=", 1)[1].split(",")]
    if only:
        what.append("models")
    if "features" in what:
        make_features()
    if "kmeans" in what:
        make_kmeans()
    if "kmeans_overlap" in what:
        make_kmeans_overlap()
    if "kmeans_latents" in what:
        make_kmeans_latents()
    if "metrics" in what:
        make_metrics()
    if "models" in what:
        make_models(only or None)
