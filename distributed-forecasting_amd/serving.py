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
"""
from __future__ import annotations

import json
import os

import numpy as np
import pandas as pd

from . import batch as B
from . import engine as E
from .forecaster import get_engine

MANIFEST = "manifest.json"


class ParamsStore:
    """Directory of per-bucket fit records, indexed by integer series keys."""

    def __init__(self, path: str, config: E.ProphetConfig | None = None):
        self.path = path
        os.makedirs(path, exist_ok=True)
        mf = os.path.join(path, MANIFEST)
        if os.path.exists(mf):
            with open(mf) as f:
                self.manifest = json.load(f)
        else:
            self.manifest = {"records": [], "config": (config or E.ProphetConfig.reference()).__dict__}
            self._write_manifest()
        self._records = {}
        self._index = None

    @property
    def config(self) -> E.ProphetConfig:
        return E.ProphetConfig(**self.manifest["config"])

    def _write_manifest(self):
        tmp = os.path.join(self.path, MANIFEST + ".tmp")
        with open(tmp, "w") as f:
            json.dump(self.manifest, f, indent=1, default=str)
        os.replace(tmp, os.path.join(self.path, MANIFEST))

    def put_batch(self, fb: B.FittedBatch, keys: np.ndarray) -> str:
        """Persist the fits of one batch; ``keys`` [n, k] integer keys."""
        return self.put_record(fb.to_record(np.asarray(keys, dtype=np.int64).reshape(fb.n, -1)))

    def put_record(self, rec: dict) -> str:
        """Persist one record (``FittedBatch.to_record`` or
        ``serialize.json_to_record`` fields, with ``keys``)."""
        if "keys" not in rec:
            raise ValueError("record needs integer 'keys' [n, k] to be indexed")
        name = f"bucket_{len(self.manifest['records']):06d}.npz"
        tmp = os.path.join(self.path, name + ".tmp.npz")
        np.savez(tmp, **rec)
        os.replace(tmp, os.path.join(self.path, name))
        self.manifest["records"].append(name)
        self._write_manifest()
        self._index = None
        return name

    def record(self, name: str) -> dict:
        if name not in self._records:
            with np.load(os.path.join(self.path, name), allow_pickle=False) as z:
                self._records[name] = {k: z[k] for k in z.files}
        return self._records[name]

    def index(self) -> dict:
        """key tuple -> (record name, row); later records win (refits)."""
        if self._index is None:
            idx = {}
            for name in self.manifest["records"]:
                keys = self.record(name)["keys"]
                for r, k in enumerate(map(tuple, keys.tolist())):
                    idx[k] = (name, r)
            self._index = idx
        return self._index

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
        yhat_lower]; each group's rows sorted by ds (Prophet.predict order)."""
        for c in ("ds", "store", "item"):
            if c not in model_input:
                raise ValueError(f"model_input must have column {c!r}")
        store = self._store
        eng = get_engine(store.config, self._device)
        idx = store.index()
        kv = np.stack([model_input["store"].to_numpy(np.int64),
                       model_input["item"].to_numpy(np.int64)], axis=1)
        ds_all = B.to_ns(model_input["ds"])
        order = np.lexsort((ds_all, kv[:, 1], kv[:, 0]))
        sk = kv[order]
        brk = np.flatnonzero(np.any(sk[1:] != sk[:-1], axis=1)) + 1
        starts = np.concatenate(([0], brk))
        ends = np.concatenate((brk, [len(order)]))
        # group the groups: same record + same (sorted) dates -> one launch
        jobs = {}
        for s, e in zip(starts, ends):
            key = tuple(sk[s].tolist())
            if key not in idx:
                raise KeyError(f"no fitted model for store={key[0]} item={key[1]} "
                               f"(run_item_{key[1]}_store_{key[0]})")
            name, row = idx[key]
            ds = ds_all[order[s:e]]
            jk = (name, ds.tobytes())
            jobs.setdefault(jk, (ds, [], []))
            jobs[jk][1].append(row)
            jobs[jk][2].append(key)
        frames = []
        for (name, _), (ds, rows, keys) in jobs.items():
            fb = B.FittedBatch.from_record(eng, store.record(name), rows)
            Tf, out = fb.predict(ds, seed=self._seed, components=False)
            n = len(rows)
            keys = np.asarray(keys, dtype=np.int64)
            fr = {"ds": np.tile(ds.astype("datetime64[ns]"), n),
                  "store": np.repeat(keys[:, 0], Tf).astype(np.int32),
                  "item": np.repeat(keys[:, 1], Tf).astype(np.int32)}
            for k in ("yhat", "yhat_upper", "yhat_lower"):
                fr[k] = out[k][:, :Tf].cpu().numpy().reshape(-1).astype(np.float32)
            frames.append(pd.DataFrame(fr))
        return pd.concat(frames, ignore_index=True)[
            ["ds", "store", "item", "yhat", "yhat_upper", "yhat_lower"]]


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
