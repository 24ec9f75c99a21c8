"""Params store + PyFunc-compatible serving model.

Reference: ``train_model`` logs each fitted Prophet as an MLflow artifact
(notebooks/prophet/02_training.py:190-196); ``ForecastStoreItemModel.predict``
looks the run up by name ``run_item_{item}_store_{store}``, sleeps
``time_between_calls``, loads the model and calls ``predict`` on the incoming
frame (notebooks/prophet/model_wrapper.py:11-73).

Here the fits of a whole bucket are one ``.npz`` record in a directory (no
pickles: plain arrays, read with ``allow_pickle=False``), and the serving
model batches every (store, item) group of its input that shares a record
and a date set into one forecast launch.

Several writers may share one store directory (torchrun ranks calling
``forecast_store_items(params_store=..., rank, world_size)``, Spark executors
running ``forecast_partitions(params_store=...)`` on a shared path): every
record gets a name unique to its writer (``rec_<time ns>_<writer>_<seq>.npz``,
written to a private temporary name and moved into place atomically), and the
index is a scan of the directory — there is no shared mutable manifest.
``manifest.json`` holds only the store's model configuration, written once
when the store is created (identical content from every creator).  Later
records win for a key that was refitted (names sort by generation: the
writer's clock unless the caller passes one, see ``ParamsStore``).
"""
from __future__ import annotations

import json
import os
import time
import uuid

import numpy as np
import pandas as pd
import torch

from . import batch as B
from . import engine as E
from .forecaster import get_engine

MANIFEST = "manifest.json"
REC_PREFIX = "rec_"
LEGACY_PREFIX = "bucket_"
# ProphetConfig fields that change what a stored fit means (its parameters,
# grid or intervals); the others (uncertainty_samples, interval_method,
# fit_mode) only steer how a caller serves or refits and may differ
FIT_FIELDS = ("growth", "n_changepoints", "changepoint_range", "yearly_seasonality",
              "weekly_seasonality", "daily_seasonality", "seasonality_mode",
              "seasonality_prior_scale", "holidays_prior_scale", "changepoint_prior_scale",
              "interval_width")


def _fit_fields(cfg: dict) -> dict:
    base = E.ProphetConfig().__dict__
    return {k: cfg.get(k, base[k]) for k in FIT_FIELDS}


class ParamsStore:
    """Directory of per-bucket fit records, indexed by integer series keys.

    Record order (which fit wins for a key that was refitted): records are
    named ``rec_<generation>_<writer>_<seq>.npz`` and sorted by name.  The
    default generation is the writer's wall clock (``time.time_ns()``), so
    with writers on several hosts the rule is only as good as their clock
    agreement; pass ``generation`` (e.g. a run counter or the training date
    as an integer) to ``put_batch`` / ``put_record`` when that matters.  Ties
    of one generation across writers break by writer id.

    Stores written by the first record format (a manifest ``records`` list of
    ``bucket_NNNNNN.npz`` files, no ``format`` key) open read-compatible:
    their listed records are indexed first, in manifest order."""

    def __init__(self, path: str, config: E.ProphetConfig | None = None, writer: str | None = None):
        self.path = path
        os.makedirs(path, exist_ok=True)
        mf = os.path.join(path, MANIFEST)
        if os.path.exists(mf):
            with open(mf) as f:
                self.manifest = json.load(f)
            if config is not None and _fit_fields(self.manifest["config"]) != _fit_fields(config.__dict__):
                raise ValueError(f"params store {path!r} holds fits made with a different "
                                 f"ProphetConfig: {self.manifest['config']}")
        else:
            self.manifest = {"config": (config or E.ProphetConfig.reference()).__dict__, "format": 2}
            tmp = os.path.join(path, f".{MANIFEST}.{uuid.uuid4().hex}")
            with open(tmp, "w") as f:
                json.dump(self.manifest, f, indent=1, default=str)
            os.replace(tmp, mf)
        # serving-side settings: the caller's, when given (fit fields agree)
        self._config = config
        self.writer = writer or f"p{os.getpid()}{uuid.uuid4().hex[:8]}"
        self._seq = 0
        self._records = {}
        self._index = None
        self._index_names = None

    @property
    def config(self) -> E.ProphetConfig:
        if self._config is not None:
            return self._config
        known = E.ProphetConfig().__dict__
        return E.ProphetConfig(**{k: v for k, v in self.manifest["config"].items() if k in known})

    @property
    def legacy_records(self) -> list:
        """Format-1 record names (manifest order), empty for a format-2 store."""
        if "format" in self.manifest:
            return []
        return list(self.manifest.get("records", []))

    def put_batch(self, fb: B.FittedBatch, keys: np.ndarray, metrics: np.ndarray | None = None,
                  generation: int | None = None) -> str:
        """Persist the fits of one batch; ``keys`` [n, k] integer keys;
        ``metrics`` [n, len(CV_METRICS)] the series' cross-validation
        metrics (what the reference logs per run, 02_training.py:187-192)."""
        rec = fb.to_record(np.asarray(keys, dtype=np.int64).reshape(fb.n, -1))
        if metrics is not None:
            from ._lib import CV_METRICS
            m = np.asarray(metrics, np.float64)
            if m.shape != (fb.n, len(CV_METRICS)):
                raise ValueError(f"metrics must be [{fb.n}, {len(CV_METRICS)}]")
            rec["cv_metrics"] = m
            rec["cv_metric_names"] = np.array(CV_METRICS)
        return self.put_record(rec, generation=generation)

    def put_record(self, rec: dict, generation: int | None = None) -> str:
        """Persist one record (``FittedBatch.to_record`` or
        ``serialize.json_to_record`` fields, with ``keys``).  Raises
        ValueError if the record was fitted under a growth, seasonality mode
        or interval width other than this store's configuration."""
        if "keys" not in rec:
            raise ValueError("record needs integer 'keys' [n, k] to be indexed")
        B.check_record_config(rec, self.config)
        gen = time.time_ns() if generation is None else int(generation)
        if gen < 0:
            raise ValueError("generation must be >= 0")
        name = f"{REC_PREFIX}{gen:020d}_{self.writer}_{self._seq:06d}.npz"
        self._seq += 1
        tmp = os.path.join(self.path, f".{name}.{uuid.uuid4().hex}.tmp.npz")
        np.savez(tmp, **rec)
        os.replace(tmp, os.path.join(self.path, name))
        self._index = None
        return name

    def record_names(self) -> list:
        """Every committed record of every writer, oldest first (format-1
        records first, in their manifest order)."""
        return self.legacy_records + sorted(
            f for f in os.listdir(self.path) if f.startswith(REC_PREFIX) and f.endswith(".npz"))

    def record(self, name: str) -> dict:
        if name not in self._records:
            with np.load(os.path.join(self.path, name), allow_pickle=False) as z:
                self._records[name] = {k: z[k] for k in z.files}
        return self._records[name]

    def index(self) -> dict:
        """key tuple -> (record name, row); later records win (refits)."""
        names = self.record_names()
        if self._index is None or names != self._index_names:
            idx = {}
            for name in names:
                keys = self.record(name)["keys"]
                for r, k in enumerate(map(tuple, keys.tolist())):
                    idx[k] = (name, r)
            self._index = idx
            self._index_names = names
        return self._index

    def metrics(self, key_cols=("store", "item")) -> pd.DataFrame:
        """The cross-validation metrics of every indexed series (its winning
        record), like the per-run metrics MLflow holds for the reference
        (02_training.py:192): [key_cols..., CV metric columns]; series fitted
        without ``cv_metrics`` are left out."""
        rows = {}
        for k, (name, r) in self.index().items():
            rec = self.record(name)
            if "cv_metrics" in rec:
                rows[k] = (tuple(str(s) for s in rec["cv_metric_names"]), rec["cv_metrics"][r])
        names = next(iter(rows.values()))[0] if rows else ()
        out = {c: np.array([k[j] for k in rows], np.int64) for j, c in enumerate(key_cols)}
        for j, m in enumerate(names):
            out[m] = np.array([v[1][j] for v in rows.values()], np.float64)
        return pd.DataFrame(out)

    def __len__(self):
        return len(self.index())


class ForecastStoreItemModel:
    """PyFunc-compatible model (model_wrapper.py:11-73) over a ParamsStore.

    ``experiment_id`` is the params-store directory (it plays the role of the
    MLflow experiment holding one run per (store, item)).  ``model_path``,
    ``dst_path`` and ``time_between_calls`` are accepted for signature
    compatibility; nothing is downloaded and nothing sleeps."""

    def __init__(self, experiment_id, model_path="model", dst_path=None,
                 time_between_calls: float = 0.5, *, device=None, seed: int = 0):
        self._experiment_id = experiment_id
        self._store = (experiment_id if isinstance(experiment_id, ParamsStore)
                       else ParamsStore(str(experiment_id)))
        self._model_path = model_path
        self._dst_path = dst_path
        self._time_between_calls = time_between_calls
        self._device = device
        self._seed = seed

    def load_context(self, context):
        """model_wrapper.py:34-40 (nothing to load eagerly)."""
        return None

    def predict(self, context, model_input: pd.DataFrame) -> pd.DataFrame:
        """model_wrapper.py:43-73, batched over every (store, item) group in
        ``model_input``.  Returns [ds, store, item, yhat, yhat_upper,
        yhat_lower]; each group's rows sorted by ds (Prophet.predict order).
        Logistic-growth stores need a ``cap`` column (UPSTREAM predict)."""
        return self._predict(model_input, True)

    def _predict(self, model_input: pd.DataFrame, guess: bool) -> pd.DataFrame:
        from .training import dense_guess
        for c in ("ds", "store", "item"):
            if c not in model_input:
                raise ValueError(f"model_input must have column {c!r}")
        store = self._store
        eng = get_engine(store.config, self._device)
        dev = torch.device("cuda", eng.device)
        logistic = store.config.growth == "logistic"
        if logistic and "cap" not in model_input:
            raise ValueError('Capacities must be supplied for logistic growth in column "cap"')
        idx = store.index()
        cols = ["ds", "store", "item", "yhat", "yhat_upper", "yhat_lower"]
        if len(model_input) == 0:
            return pd.DataFrame({c: pd.Series(dtype=("datetime64[ns]" if c == "ds" else np.int32
                                                     if c in ("store", "item") else np.float32))
                                 for c in cols})

        def lookup(key):
            if key not in idx:
                raise KeyError(f"no fitted model for store={key[0]} item={key[1]} "
                               f"(run_item_{key[1]}_store_{key[0]})")
            return idx[key]

        # group the groups: same record + same (sorted) dates -> one launch
        jobs = {}
        # grouped input in key order, every group on the same dates: no
        # per-group date handling (the usual scoring frame).  The layout is
        # read off the first group; the O(rows) checks run while the GPU works
        dense = dense_guess(model_input, ["store", "item"], value="cap" if logistic else None) \
            if guess else None
        verify = None
        if dense is not None:
            gkeys, ds0, capm, verify = dense
            verify.start()
            for g, key in enumerate(map(tuple, gkeys.tolist())):
                try:
                    name, row = lookup(key)
                except KeyError:
                    if verify():
                        raise
                    return self._predict(model_input, False)
                j = jobs.setdefault(name, (ds0, [], [], []))
                j[1].append(row)
                j[2].append(key)
                if logistic:
                    j[3].append(capm[g])
        else:
            st_col = model_input["store"].to_numpy(np.int64)
            it_col = model_input["item"].to_numpy(np.int64)
            ds_all = B.to_ns(model_input["ds"])
            cap_all = model_input["cap"].to_numpy(np.float64) if logistic else None
            n_in = st_col.shape[0]
            # rows ordered by (store, item, ds); an input already in that
            # order is not sorted again
            code = (st_col - int(st_col.min())) * (int(it_col.max()) - int(it_col.min()) + 1) + \
                (it_col - int(it_col.min()))
            same = code[1:] == code[:-1]
            if bool(np.all(code[1:] >= code[:-1])) and bool(np.all(~same | (ds_all[1:] >= ds_all[:-1]))):
                order = np.arange(n_in)
                sc = code
            else:
                order = np.lexsort((ds_all, code))
                sc = code[order]
            brk = np.flatnonzero(sc[1:] != sc[:-1]) + 1
            starts = np.concatenate(([0], brk))
            ends = np.concatenate((brk, [len(order)]))
            for s, e in zip(starts, ends):
                key = (int(st_col[order[s]]), int(it_col[order[s]]))
                name, row = lookup(key)
                ds = ds_all[order[s:e]]
                j = jobs.setdefault((name, ds.tobytes()), (ds, [], [], []))
                j[1].append(row)
                j[2].append(key)
                if logistic:
                    j[3].append(cap_all[order[s:e]])
        # launch every job, D2H into pinned memory asynchronously, then
        # build the key / date columns while the GPU works
        launched = []
        for jk, (ds, rows, keys, caps) in jobs.items():
            name = jk if isinstance(jk, str) else jk[0]
            fb = B.FittedBatch.from_record(eng, store.record(name), rows)
            Tf, out = fb.predict(ds, seed=self._seed, components=False,
                                 cap=np.stack(caps) if logistic else None)
            blk = torch.stack([out[k][:, :Tf] for k in ("yhat", "yhat_upper", "yhat_lower")])
            host = torch.empty(blk.shape, dtype=blk.dtype, pin_memory=True)
            host.copy_(blk, non_blocking=True)
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(dev))
            launched.append((ds, keys, Tf, host, done))
        if verify is not None and not verify():
            return self._predict(model_input, False)   # not the dense layout
        frames = []
        for ds, keys, Tf, host, done in launched:
            n = len(keys)
            keys = np.asarray(keys, dtype=np.int64)
            fr = {"ds": np.tile(np.asarray(ds, np.int64).view("datetime64[ns]"), n),
                  "store": np.repeat(keys[:, 0].astype(np.int32), Tf),
                  "item": np.repeat(keys[:, 1].astype(np.int32), Tf)}
            frames.append((fr, host, done))
        for fr, host, done in frames:
            done.synchronize()
            h = host.numpy()
            for j, k in enumerate(("yhat", "yhat_upper", "yhat_lower")):
                fr[k] = h[j].reshape(-1)
        frames = [f for f, _, _ in frames]
        return pd.DataFrame({c: (frames[0][c] if len(frames) == 1 else
                                 np.concatenate([f[c] for f in frames])) for c in cols}, copy=False)


_REGISTERED = {}


def register_model(model: ForecastStoreItemModel, name: str = "ForecastingModelUDF"):
    """Stand-in for the MLflow model registry entry 04_inference.py:10-13 reads."""
    _REGISTERED[name] = model


def predict_udf(history_pd: pd.DataFrame, model: ForecastStoreItemModel | None = None,
                model_name: str = "ForecastingModelUDF") -> pd.DataFrame:
    """notebooks/prophet/04_inference.py:4-16: serve one group's frame with
    the registered model (or ``model``)."""
    if model is None:
        if model_name not in _REGISTERED:
            raise KeyError(f"no registered model {model_name!r}: call register_model first")
        model = _REGISTERED[model_name]
    return model.predict(None, history_pd)
