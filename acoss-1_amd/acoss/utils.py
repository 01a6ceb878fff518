"""General helpers of the benchmark, same names and behaviour as acoss/utils.py of the
reference (file:line cited per function). Only the dataset-annotation side is kept here;
audio batching for feature extraction belongs to the extractor, which is out of scope."""
import json
import logging
import os
import time

import pandas as pd

ACOSS_PATH = os.path.dirname(os.path.abspath(__file__))
# acoss/utils.py:15-21 — the two annotation CSVs that ship with the package
DA_TACOS_BENCHMARK_CSV = os.path.join(ACOSS_PATH, "data/da-tacos_benchmark_subset.csv")
COVERS_80_CSV = os.path.join(ACOSS_PATH, "data/covers80_annotations.csv")


def log(log_file):
    """Logger writing to `log_file` and the console (acoss/utils.py:24-35)."""
    logger = logging.getLogger(__name__)
    logger.setLevel(logging.DEBUG)
    fmt = logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    if not any(isinstance(h, logging.FileHandler) and getattr(h, "baseFilename", None) == os.path.abspath(log_file)
               for h in logger.handlers):
        fh = logging.FileHandler(log_file)
        fh.setFormatter(fmt)
        logger.addHandler(fh)
        ch = logging.StreamHandler()
        ch.setFormatter(fmt)
        logger.addHandler(ch)
    return logger


def timeit(method):
    """Timing decorator (acoss/utils.py:38-50): prints ms, or records into kw['log_time']."""
    def timed(*args, **kw):
        t0 = time.time()
        result = method(*args, **kw)
        ms = (time.time() - t0) * 1000
        if "log_time" in kw:
            kw["log_time"][kw.get("log_name", method.__name__.upper())] = int(ms)
        else:
            print("%r - runtime : %2.2f ms" % (method.__name__, ms))
        return result
    return timed


def read_txt_file(txt_file):
    """Lines of a text file without their newline (acoss/utils.py:53-57)."""
    with open(txt_file) as f:
        return [line.replace("\n", "") for line in f.readlines()]


def savelist_to_file(path_list, filename):
    """One item per line (acoss/utils.py:60-64)."""
    with open(filename, "w") as f:
        for item in path_list:
            f.write("%s\n" % item)


def create_dataset_filepaths(dataset_csv, root_audio_dir, file_format=".mp3"):
    """root_audio_dir + work_id + "/" + track_id + file_format for every CSV row
    (acoss/utils.py:87-102). The CSV must have exactly the columns work_id, track_id;
    anything else raises IOError. Paths are built by plain string concatenation, as in the
    reference, so root_audio_dir needs its trailing slash."""
    dataset = pd.read_csv(dataset_csv, dtype=str)
    for key in dataset.keys().tolist():
        if key not in ("work_id", "track_id"):
            raise IOError("Wrong input dataset csv annotation file '%s'. Expected a csv file with the columns of key "
                          "'work_id', 'track_id'" % dataset_csv)
    return [root_audio_dir + str(w) + "/" + str(t) + file_format for w, t in zip(dataset.work_id, dataset.track_id)]


def da_tacos_metadata_to_acoss_csv(datacos_metadata_json, output_csv):
    """Da-TACOS metadata json {work_id: {perf_id: ...}} -> acoss CSV (acoss/utils.py:105-116)."""
    with open(datacos_metadata_json) as f:
        meta = json.load(f)
    rows = [(w, p) for w in meta for p in meta[w]]
    pd.DataFrame({"work_id": [w for w, _ in rows], "track_id": [p for _, p in rows]}).to_csv(output_csv, index=False)


def generate_covers80_acoss_csv(covers80_audio_data_path, output_csv):
    """covers80 folder layout work/track.mp3 -> acoss CSV (acoss/utils.py:119-131)."""
    works, tracks = [], []
    for work in os.listdir(covers80_audio_data_path):
        wp = os.path.join(covers80_audio_data_path, work)
        if os.path.isdir(wp):
            for t in os.listdir(wp):
                if t.endswith(".mp3"):
                    works.append(work)
                    tracks.append(t.replace(".mp3", ""))
    pd.DataFrame({"work_id": works, "track_id": tracks}).to_csv(output_csv, index=False)
