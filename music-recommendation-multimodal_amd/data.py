"""The two-tower step's caller: the batch contract of the reference's MultimodalDataset
(SURVEY §8(f) rank 1).  ``src/data/dataset.py`` is missing from the reference snapshot
(SURVEY §0.2), so the contract is the one its call sites imply:

* constructor ``MultimodalDataset(interactions_df, item_id_mapper, img_dir, audio_dir=None,
  text_data=None, tokenizer=None, max_seq_len=50, encoders=None)``
  (train.py:223-241, inference.py:80-87, evaluate_metrics.py:41-49, test_dataset_loading.py:37);
* ``.encoders`` = {'gender_encoder', 'country_encoder' (``classes_``), 'genre_encoder'
  (``categories_``), 'scaler' (``mean_``)} and ``get_encoders()`` (train.py:240,256,280-285;
  scripts/inspect_encoders.py:13-19); the fitted objects are scikit-learn's, as in the
  reference's ``encoders.pkl``;
* ``.tabular_data`` (``shape[1]`` = T: the 14 Spotify numerics standardised + one-hot
  ``track_genre``, dataset.tex:10-11), ``.user_groups`` (user -> chronological track list,
  overridable: train.py:245-246), ``.interactions_df`` with ``gender_idx`` / ``country_idx``
  (inference.py:263-264), ``.item_id_mapper``, ``.img_dir``, ``.audio_dir``, ``.text_data``,
  ``.tokenizer``;
* item ``i`` = interaction row ``i``: ``history_ids`` = the user's tracks before it
  (``seq_idx`` = per-user cumcount in timestamp order, evaluate_metrics.py:237), the last
  ``max_seq_len`` (inference.py:254-259), right-padded (user_tower.py:122-132 takes the last
  valid row); keys of two_tower.py:68-142 plus ``target_id`` / ``user_id`` / ``user_idx``.

MI355X layout decision: items carry RAW modalities (uint8 HWC cover, the stored mel or the
waveform); ``DeviceCollator`` stages a batch to HBM and runs the HIP preprocessing kernels
(``preprocess.py``) there — the reference resized / normalised per item on CPU workers.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional

import numpy as np
import torch
from torch import Tensor

NUMERIC_FEATURES = ("popularity", "duration_ms", "danceability", "energy", "key", "loudness",
                    "mode", "speechiness", "acousticness", "instrumentalness", "liveness",
                    "valence", "tempo", "time_signature")          # dataset.tex:10 (14 numerics)
MISSING_COVER = (300, 300)                                        # Spotify 300 px covers (dataset.tex:36)


def _label_fit(values):
    from sklearn.preprocessing import LabelEncoder
    return LabelEncoder().fit(values)


def fit_encoders(df) -> Dict[str, object]:
    """The reference's encoders.pkl content, fitted on an interactions frame."""
    from sklearn.preprocessing import OneHotEncoder, StandardScaler
    tracks = df.drop_duplicates("track_id")
    enc = {
        "gender_encoder": _label_fit(df["gender"].fillna("unknown").astype(str)),
        "country_encoder": _label_fit(df["country"].fillna("unknown").astype(str)),
        "genre_encoder": OneHotEncoder(handle_unknown="ignore", sparse_output=False).fit(
            tracks[["track_genre"]].fillna("unknown").astype(str)),
        "scaler": StandardScaler().fit(tracks[list(NUMERIC_FEATURES)].astype(np.float64).values),
    }
    return enc


def _encode(le, values) -> np.ndarray:
    """LabelEncoder.transform with unseen labels -> 0."""
    lut = {c: i for i, c in enumerate(le.classes_)}
    return np.array([lut.get(v, 0) for v in values], dtype=np.int64)


class MultimodalDataset(torch.utils.data.Dataset):
    def __init__(self, interactions_df, item_id_mapper: Dict[str, int], img_dir: Optional[str] = None,
                 audio_dir: Optional[str] = None, text_data: Optional[Dict[str, str]] = None,
                 tokenizer=None, max_seq_len: int = 50, encoders: Optional[Dict[str, object]] = None,
                 text_max_len: int = 256, mel_shape=(128, 128)):
        import pandas as pd
        df = interactions_df.copy()
        if "timestamp" in df.columns:
            df["timestamp"] = pd.to_datetime(df["timestamp"], utc=True)
            df = df.sort_values("timestamp", kind="stable")
        if "seq_idx" not in df.columns:
            df["seq_idx"] = df.groupby("user_id").cumcount().astype(int)
        self.encoders = encoders if encoders is not None else fit_encoders(df)
        df["gender_idx"] = _encode(self.encoders["gender_encoder"], df["gender"].fillna("unknown").astype(str))
        df["country_idx"] = _encode(self.encoders["country_encoder"], df["country"].fillna("unknown").astype(str))
        self.interactions_df = df.reset_index(drop=True)
        self.item_id_mapper = item_id_mapper
        self.img_dir, self.audio_dir = img_dir, audio_dir
        self.text_data = text_data if text_data is not None else {}
        self.tokenizer = tokenizer
        self.max_seq_len, self.text_max_len = max_seq_len, text_max_len
        self.mel_shape = tuple(mel_shape)
        self.user_groups: Dict[str, List[str]] = df.groupby("user_id", sort=False)["track_id"].apply(list).to_dict()
        users = sorted(self.user_groups)
        self._user_index = {u: i for i, u in enumerate(users)}
        tracks = df.drop_duplicates("track_id")
        num = self.encoders["scaler"].transform(tracks[list(NUMERIC_FEATURES)].astype(np.float64).values)
        gen = self.encoders["genre_encoder"].transform(tracks[["track_genre"]].fillna("unknown").astype(str))
        self.tabular_data = np.concatenate([num, gen], axis=1).astype(np.float32)
        self._track_row = {t: i for i, t in enumerate(tracks["track_id"].tolist())}
        # columns as numpy for a cheap __getitem__
        self._uid = self.interactions_df["user_id"].to_numpy()
        self._tid = self.interactions_df["track_id"].to_numpy()
        self._seq = self.interactions_df["seq_idx"].to_numpy()
        self._gender = self.interactions_df["gender_idx"].to_numpy()
        self._country = self.interactions_df["country_idx"].to_numpy()

    def get_encoders(self) -> Dict[str, object]:
        return self.encoders

    def __len__(self) -> int:
        return len(self.interactions_df)

    # ---------------------------------------------------------------- per-item pieces
    def history(self, user_id: str, seq_idx: int):
        hist = self.user_groups.get(user_id, [])[:int(seq_idx)][-self.max_seq_len:]
        ids = np.zeros(self.max_seq_len, dtype=np.int64)
        mask = np.zeros(self.max_seq_len, dtype=np.int64)
        n = len(hist)
        if n:
            ids[:n] = [self.item_id_mapper.get(t, 0) for t in hist]
            mask[:n] = 1
        return ids, mask

    def cover(self, track_id: str) -> np.ndarray:
        """Raw uint8 HWC cover (zeros when absent; resized to 300 x 300 if stored otherwise)."""
        if self.img_dir:
            path = os.path.join(self.img_dir, f"{track_id}.jpg")
            if os.path.exists(path):
                from PIL import Image
                with Image.open(path) as im:
                    im = im.convert("RGB")
                    if im.size != MISSING_COVER[::-1]:
                        im = im.resize(MISSING_COVER[::-1], Image.BILINEAR)
                    return np.asarray(im, dtype=np.uint8)
        return np.zeros(MISSING_COVER + (3,), dtype=np.uint8)

    def audio(self, track_id: str) -> np.ndarray:
        """The stored mel [n_mels, T] (already in [0, 1]) or a 1-D waveform; zeros when absent."""
        if self.audio_dir:
            path = os.path.join(self.audio_dir, f"{track_id}.npy")
            if os.path.exists(path):
                return np.load(path, allow_pickle=False).astype(np.float32)
        return np.zeros(self.mel_shape, dtype=np.float32)

    def text(self, track_id: str):
        S = self.text_max_len
        if self.tokenizer is None or track_id not in self.text_data:
            return np.zeros(S, dtype=np.int64), np.zeros(S, dtype=np.int64)
        enc = self.tokenizer(self.text_data[track_id], max_length=S, padding="max_length", truncation=True)
        return np.asarray(enc["input_ids"], dtype=np.int64), np.asarray(enc["attention_mask"], dtype=np.int64)

    def __getitem__(self, idx: int) -> Dict[str, object]:
        uid, tid = self._uid[idx], self._tid[idx]
        hist, hmask = self.history(uid, self._seq[idx])
        ids, amask = self.text(tid)
        row = self._track_row.get(tid)
        tab = self.tabular_data[row] if row is not None else np.zeros(self.tabular_data.shape[1], np.float32)
        return {
            "user_id": uid,
            "user_idx": np.int64(self._user_index.get(uid, 0)),
            "history_ids": hist, "history_mask": hmask,
            "user_gender": np.int64(self._gender[idx]), "user_country": np.int64(self._country[idx]),
            "target_id": np.int64(self.item_id_mapper.get(tid, 0)),
            "target_image_u8": self.cover(tid),
            "target_audio_raw": self.audio(tid),
            "target_input_ids": ids, "target_attention_mask": amask,
            "target_tabular": tab,
        }


def collate(items: List[Dict[str, object]]) -> Dict[str, object]:
    """Host collation into pinned tensors (DataLoader ``collate_fn``)."""
    out: Dict[str, object] = {"user_id": [it["user_id"] for it in items]}
    for k in items[0]:
        if k == "user_id":
            continue
        if k == "target_audio_raw":
            shapes = {np.shape(it[k]) for it in items}
            if len(shapes) != 1:
                raise ValueError(f"collate: audio items of different shapes {sorted(shapes)}")
        t = torch.from_numpy(np.stack([np.asarray(it[k]) for it in items]))
        out[k] = t.pin_memory() if torch.cuda.is_available() else t
    return out


class DeviceCollator:
    """Stage a collated host batch to the GPU and run the modality transforms there: covers
    through ``CoverTransform`` (NCHW fp32 ``target_image``), waveforms through ``MelSpectrogram``
    (stored mels pass through).  Copies are non-blocking on the current stream."""

    def __init__(self, device="cuda", image_size: int = 224, mel: Optional[object] = None):
        from . import preprocess as P
        self.device = torch.device(device)
        self.cover = P.CoverTransform(image_size)
        self.mel = mel if mel is not None else P.MelSpectrogram(device=device)

    def __call__(self, batch: Dict[str, object]) -> Dict[str, object]:
        out: Dict[str, object] = {}
        for k, v in batch.items():
            out[k] = v.to(self.device, non_blocking=True) if isinstance(v, Tensor) else v
        out["target_image"] = self.cover(out.pop("target_image_u8").contiguous())
        a = out.pop("target_audio_raw")
        out["target_audio"] = self.mel(a.float().contiguous()) if a.dim() == 2 else a.float().unsqueeze(1)
        return out


class DevicePrefetcher:
    """Overlap the next batch's H2D copy and preprocessing with the current step: batches are
    produced on a side HIP stream and handed over with an event (double buffering)."""

    def __init__(self, loader: Iterable, collator: DeviceCollator):
        self.loader, self.collator = loader, collator
        self.stream = torch.cuda.Stream()

    def __iter__(self):
        it = iter(self.loader)
        nxt = self._stage(it)
        while nxt is not None:
            cur, ev = nxt
            torch.cuda.current_stream().wait_event(ev)
            for v in cur.values():
                if isinstance(v, Tensor):
                    v.record_stream(torch.cuda.current_stream())
            nxt = self._stage(it)
            yield cur

    def _stage(self, it):
        try:
            host = next(it)
        except StopIteration:
            return None
        with torch.cuda.stream(self.stream):
            dev = self.collator(host)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return dev, ev


# ------------------------------------------------------------------ synthetic data
def synthetic_interactions(n_users: int = 100, n_items: int = 1000, n_events: int = 5000,
                           n_genres: int = 12, seed: int = 0):
    """An interactions frame with the merged Last.fm x Spotify columns (notebook 04's
    ``df_sampled``: user_id, gender, country, timestamp, track_id, ..., track_genre)."""
    import pandas as pd
    rng = np.random.default_rng(seed)
    users = [f"user_{i:06d}" for i in range(n_users)]
    tracks = [f"trk{i:019d}" for i in range(n_items)]
    gender = rng.choice(["m", "f", "n"], n_users)
    country = rng.choice([f"country_{i}" for i in range(20)], n_users)
    u = rng.integers(0, n_users, n_events)
    t = rng.integers(0, n_items, n_events)
    ts = pd.Timestamp("2008-01-01", tz="UTC") + pd.to_timedelta(rng.integers(0, 10 ** 8, n_events), unit="s")
    item_feat = {
        "popularity": rng.integers(0, 100, n_items), "duration_ms": rng.integers(90_000, 400_000, n_items),
        "danceability": rng.random(n_items), "energy": rng.random(n_items),
        "key": rng.integers(0, 12, n_items), "loudness": rng.normal(-8, 3, n_items),
        "mode": rng.integers(0, 2, n_items), "speechiness": rng.random(n_items) * 0.3,
        "acousticness": rng.random(n_items), "instrumentalness": rng.random(n_items),
        "liveness": rng.random(n_items), "valence": rng.random(n_items),
        "tempo": rng.normal(120, 25, n_items), "time_signature": rng.integers(3, 6, n_items),
    }
    genres = np.array([f"genre_{g}" for g in range(n_genres)])[rng.integers(0, n_genres, n_items)]
    df = pd.DataFrame({
        "user_id": np.array(users)[u], "gender": gender[u], "country": country[u], "timestamp": ts,
        "track_id": np.array(tracks)[t], "artist_name": [f"artist {i % 97}" for i in t],
        "track_name": [f"track {i}" for i in t], "album_name": [f"album {i % 311}" for i in t],
        **{k: v[t] for k, v in item_feat.items()}, "explicit": rng.random(n_events) < 0.1,
        "track_genre": genres[t],
    })
    return df


def item_id_mapper_from(df) -> Dict[str, int]:
    """train.py:150-152: 1-based ids in order of first appearance."""
    return {tid: i + 1 for i, tid in enumerate(df["track_id"].unique())}


def text_data_from(df) -> Dict[str, str]:
    """train.py:178-183: "artist - track (album)" per track."""
    u = df.drop_duplicates("track_id")
    texts = (u["artist_name"].fillna("") + " - " + u["track_name"].fillna("") + " (" +
             u["album_name"].fillna("") + ")")
    return dict(zip(u["track_id"], texts))
