"""Per-track feature files: the dict the reference reads with deepdish (`dd.io.load`,
acoss/algorithms/algorithm_template.py:90; written by acoss/extractors.py:114).

Keys (README.md:93-114): 'hpcp', 'crema', 'chroma_cens' (n, 12) float32, 'mfcc_htk'
(n_coeffs, n), 'madmom_features' {'onsets': int64, ...}, 'label', 'track_id', ...

Readers, in order:
  1. `<path>` itself when it is HDF5 and h5py is importable (deepdish's layout: datasets for
     arrays, groups for nested dicts, scalar/str datasets or attributes for the rest);
  2. the same path with the suffix `.npz` (np.load, allow_pickle=False), nested keys
     flattened as 'madmom_features/onsets'. This image has neither h5py nor PyTables, so the
     tests and the synthetic datasets use this form (`save_features`).
An HDF5 dataset compressed with a filter h5py cannot decode (deepdish's default blosc, without
the plugin) raises IOError naming the filter and the one-line .npz conversion.
"""
import os

import numpy as np


def _npz_path(path):
    root, ext = os.path.splitext(path)
    return root + ".npz" if ext != ".npz" else path


def _unflatten(flat):
    out = {}
    for key, val in flat.items():
        parts = key.split("/")
        d = out
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        if isinstance(val, np.ndarray) and val.ndim == 0:
            val = val.item()
        d[parts[-1]] = val
    return out


def _flatten(feats, prefix=""):
    flat = {}
    for k, v in feats.items():
        name = prefix + str(k)
        if isinstance(v, dict):
            flat.update(_flatten(v, name + "/"))
        else:
            flat[name] = np.asarray(v)
    return flat


# HDF5 filter codes h5py cannot decode without a plugin (deepdish writes through PyTables with
# blosc by default)
_FILTER_NAMES = {32001: "blosc", 32004: "lz4", 32008: "bitshuffle", 32015: "zstd", 307: "bzip2"}

CONVERT_RECIPE = ("convert the file once on a machine with deepdish: `import deepdish as dd; "
                  "from acoss.features_io import save_features; save_features(path, dd.io.load(path))` "
                  "(writes the .npz twin this reader takes), or install the filter plugin (hdf5plugin)")


def _missing_filters(h5py, ds):
    """Names of the dataset's HDF5 filters that this h5py/libhdf5 cannot apply."""
    out = []
    plist = ds.id.get_create_plist()
    for i in range(plist.get_nfilters()):
        code, _, _, name = plist.get_filter(i)
        if not h5py.h5z.filter_avail(code):
            nm = name.decode(errors="replace") if isinstance(name, bytes) else str(name)
            out.append("%s (filter %d)" % (_FILTER_NAMES.get(code, nm or "unknown"), code))
    return out


def _read_dataset(h5py, path, key, ds):
    """ds[()], raising IOError that names the filter and the .npz conversion when the read fails
    on a compression filter this libhdf5 lacks (h5py's own message names only a plugin dir)."""
    try:
        return ds[()]
    except OSError as e:
        missing = _missing_filters(h5py, ds)
        if missing:
            raise IOError("%s: dataset '%s' is compressed with %s, which this h5py cannot decode; %s"
                          % (path, key, ", ".join(missing), CONVERT_RECIPE)) from e
        raise


def _load_h5(path):
    import h5py  # optional

    def walk(g):
        d = {}
        for k, v in g.items():
            if isinstance(v, h5py.Group):
                d[k] = walk(v)
            else:
                a = _read_dataset(h5py, path, v.name, v)
                d[k] = a.decode() if isinstance(a, bytes) else a
        for k, v in g.attrs.items():
            if k not in d and not k.startswith("DEEPDISH") and not k.startswith("CLASS"):
                d[k] = v.decode() if isinstance(v, bytes) else v
        return d

    with h5py.File(path, "r") as f:
        return walk(f)


def save_h5(path, mats, h5py):
    """A dict of arrays as an HDF5 file in deepdish's dict layout (one dataset per key under
    the root group), for the reference's '<prefix>_Ds.h5' (algorithm_template.py:193)."""
    with h5py.File(path, "w") as f:
        f.attrs["DEEPDISH_IO_VERSION"] = 12
        for k, v in mats.items():
            f.create_dataset(str(k), data=np.asarray(v))


def load_features(path, keys=None):
    """Feature dict of one track; IOError if no readable file exists. keys: read only these
    top-level entries (e.g. the chroma type and 'label'); None reads the whole dict."""
    p = _npz_path(path)
    if os.path.exists(path) and not path.endswith(".npz"):
        try:
            d = _load_h5(path)
            return d if keys is None else {k: d[k] for k in keys if k in d}
        except ImportError:
            pass
        except IOError:
            if not os.path.exists(p):  # an undecodable filter and no converted twin
                raise
    if os.path.exists(p):
        with np.load(p, allow_pickle=False) as z:
            names = z.files if keys is None else [k for k in z.files if k.split("/")[0] in keys]
            return _unflatten({k: z[k] for k in names})
    raise IOError("no readable feature file for %s (looked for HDF5 with h5py, and %s)" % (path, p))


def _h5_readable():
    try:
        import h5py  # noqa: F401
        return True
    except ImportError:
        return False


def cache_readable(path):
    """True when load_features(path) has a file to read: the .npz twin, or the HDF5 file itself
    with h5py importable."""
    return os.path.exists(_npz_path(path)) or (os.path.exists(path) and not path.endswith(".npz") and _h5_readable())


def load_many(paths, keys=None, workers=None):
    """load_features over many tracks, results in input order. The .npz twins are read by the
    native reader (acoss_npz_index / acoss_npz_read: zip directory, .npy headers and data on
    `workers` std::threads inside one C call, no GIL; 15,000 files took 12-17 s through np.load on
    a 16-thread pool, which the GIL serialised). Paths whose deepdish .h5 is readable (h5py
    present) and the rare file the native reader refuses go through load_features."""
    if workers is None:
        workers = min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1)
    h5 = _h5_readable()
    native_idx, npz = [], []
    for i, p in enumerate(paths):
        twin = _npz_path(p)
        if (h5 and os.path.exists(p) and not p.endswith(".npz")) or not os.path.exists(twin):
            continue
        native_idx.append(i)
        npz.append(twin)
    out = [None] * len(paths)
    if native_idx:
        try:
            from . import _lib
            got = _lib.npz_read_many(npz, keys, n_threads=workers)
        except (IOError, OSError, ImportError, RuntimeError):
            got = None  # a file the native reader refuses: np.load says what is wrong with it
        if got is not None:
            for i, flat in zip(native_idx, got):
                out[i] = _unflatten(flat)
    rest = [i for i in range(len(paths)) if out[i] is None]
    if len(rest) > 1 and workers > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=workers) as ex:
            for i, d in zip(rest, ex.map(lambda i: load_features(paths[i], keys), rest)):
                out[i] = d
    else:
        for i in rest:
            out[i] = load_features(paths[i], keys)
    return out


def save_features(path, feats):
    """Write `feats` as the .npz twin of `path` (creates the directory). Written to a temporary
    name and renamed into place, so ranks caching the same song (EarlyFusion's block features)
    never leave a torn file for each other."""
    p = _npz_path(path)
    os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
    tmp = "%s.tmp%d.npz" % (p[:-4], os.getpid())
    np.savez(tmp, **_flatten(feats))
    os.replace(tmp, p)
    return p
