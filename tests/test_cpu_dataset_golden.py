"""Data pipeline pinned against the reference's own dataset module.

tests/golden/dataset.npz holds the raw rows of a small database in the reference schema
(database.py:28-47 + the l0..l4 load columns dataset.py:30 reads) and what the reference's
``dataset.get_train_data`` / ``get_validation_data`` / ``get_test_data`` (dataset.py:61-95 ->
database.get_data database.py:128-147 -> process_dataframe dataset.py:39-54) and
``dataframe_to_dataset`` (dataset.py:98-103) returned for it (tests/golden/make_golden.py ran them).
Here the same rows go into a fresh SQLite file and p2pmicrogrid_amd.dataset must return the
same frames, bit for bit."""
import os
import sqlite3

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden", "dataset.npz")


@pytest.fixture()
def reference_db(tmp_path, monkeypatch):
    g = np.load(GOLD)
    path = str(tmp_path / "ref.db")
    con = sqlite3.connect(path)
    cur = con.cursor()
    cur.execute("CREATE TABLE environment (date text NOT NULL, time text NOT NULL, utc text NOT NULL, "
                "temperature real, cloud_cover real, humidity real, irradiation real, pv real, "
                "PRIMARY KEY (date, time, utc))")
    cur.execute("CREATE TABLE load (date text NOT NULL, time text NOT NULL, utc text NOT NULL, load_0 real, "
                "l0 real, l1 real, l2 real, l3 real, l4 real, PRIMARY KEY (date, time, utc))")
    cur.executemany("INSERT INTO environment VALUES (?,?,?,?,?,?,?,?)",
                    [(*map(str, k), *map(float, v)) for k, v in zip(g["env_rows"], g["env_vals"])])
    cur.executemany("INSERT INTO load VALUES (?,?,?,?,?,?,?,?,?)",
                    [(*map(str, k), *map(float, v)) for k, v in zip(g["load_rows"], g["load_vals"])])
    con.commit()
    con.close()
    monkeypatch.setenv("P2PMG_DB", path)
    return g


@pytest.mark.parametrize("split", ["train", "validation", "test"])
def test_get_data_matches_reference(reference_db, split):
    from p2pmicrogrid_amd import dataset as ds
    g = reference_db
    env_df, agent_dfs = {"train": ds.get_train_data, "validation": ds.get_validation_data,
                         "test": ds.get_test_data}[split]()
    assert list(env_df.columns) == list(g[f"{split}_env_cols"])
    assert np.array_equal(env_df.index.to_numpy(), g[f"{split}_index"])
    assert np.array_equal(env_df.to_numpy(dtype=np.float64), g[f"{split}_env"])
    assert len(agent_dfs) == 5
    assert all(list(a.columns) == list(g[f"{split}_agent_cols"]) for a in agent_dfs)
    assert np.array_equal(np.stack([a.to_numpy(dtype=np.float64) for a in agent_dfs]), g[f"{split}_agents"])


def test_dataframe_to_dataset_matches_reference(reference_db):
    from p2pmicrogrid_amd import dataset as ds
    env_df, _ = ds.get_train_data()
    d = ds.dataframe_to_dataset(env_df)
    assert d.data.dtype == np.float32
    assert np.array_equal(d.data, reference_db["train_ds_x"])
    assert np.array_equal(d.rolled, reference_db["train_ds_rolled"])


def test_shared_scenario_inputs_equal_serial_generation():
    """bench.py generates configs[3]'s year of inputs with a worker pool into shared memory
    (dataset.SharedScenarioInputs): the same arrays bit for bit as scenario_batch + apply_asset_mix,
    for a shard that starts and ends inside generator blocks."""
    from p2pmicrogrid_amd.dataset import SharedScenarioInputs, apply_asset_mix, asset_mix, scenario_batch
    S, N, T, first = 300, 3, 200, 200
    mix = asset_mix(S, N, first_scenario=first, battery_j=36e6)
    ref = apply_asset_mix(scenario_batch(S, N, T, first_scenario=first), mix)
    with SharedScenarioInputs(S, N, T, workers=2, first_scenario=first, mix=mix) as sh:
        got = sh.inputs
        for k in ("time", "t_out", "load_w", "pv_w", "max_in", "t_in0", "t_m0", "load_ratings", "pv_ratings"):
            a, b = getattr(ref, k), getattr(got, k)
            assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b), k
        del got, a, b
