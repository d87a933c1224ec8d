"""database.py sinks / source with the reference's schema (database.py:28-81, 128-147, 198-312)
and dataset.get_data reading a database the way dataset.py:61-80 does."""
import sqlite3

import numpy as np


def _make_db(path, days=(11, 12, 18)):
    from p2pmicrogrid_amd import database as db
    con = sqlite3.connect(path)
    cur = con.cursor()
    db.create_tables(cur)
    cur.execute("ALTER TABLE load ADD COLUMN l0 real")  # the reference's data carry l0..l4 (dataset.py:30)
    for k in range(1, 5):
        cur.execute(f"ALTER TABLE load ADD COLUMN l{k} real")
    rs = np.random.RandomState(0)
    rows_e, rows_l = [], []
    for d in days:
        for slot in range(96):
            date, tm = f"2021-10-{d:02d}", f"{slot // 4:02d}:{15 * (slot % 4):02d}:00"
            rows_e.append((date, tm, "+00:00", float(rs.normal(10, 3)), 0.5, 0.7, 0.0, float(max(0, np.sin(slot / 30)))))
            rows_l.append((date, tm, "+00:00", 0.0, *[float(rs.rand() + 0.1) for _ in range(5)]))
    cur.executemany("INSERT INTO environment VALUES (?,?,?,?,?,?,?,?)", rows_e)
    cur.executemany("INSERT INTO load VALUES (?,?,?,?,?,?,?,?,?)", rows_l)
    con.commit()
    return con


def test_get_data_reads_reference_schema(tmp_path, monkeypatch):
    from p2pmicrogrid_amd import dataset as ds
    path = str(tmp_path / "data.db")
    _make_db(path).close()
    monkeypatch.setenv("P2PMG_DB", path)
    env_df, agent_dfs = ds.get_train_data()  # days 11..17: only 11 and 12 exist
    assert list(env_df.columns) == ["time", "temperature"] and len(env_df) == 192
    assert np.allclose(env_df["time"].values[:4], [0, 1 / 96, 2 / 96, 3 / 96])
    assert len(agent_dfs) == 5 and list(agent_dfs[0].columns) == ["load", "pv"]
    assert agent_dfs[2]["load"].max() == 1.0 and agent_dfs[0]["pv"].max() == 1.0
    v_env, _ = ds.get_validation_data()
    assert set(v_env["day"]) == {18} and len(v_env) == 96


def test_result_sinks_roundtrip(tmp_path):
    from p2pmicrogrid_amd import database as db
    con = db.get_connection(str(tmp_path / "r.db"))
    db.create_tables(con.cursor())
    db.log_test_results(con, "2-multi", 1, [8] * 3, [0.0, 0.01, 0.02], [1, 2, 3], [0, 0, 1], [21, 21.1, 21.2],
                        [0, 1500, 3000], [0.1, 0.2, 0.3], "tabular")
    db.log_validation_results(con, "2-multi", 0, [18] * 2, [0.0, 0.01], [1, 2], [0, 0], [21, 21], [0, 0], [0, 0],
                              "tabular")
    db.log_rounds_decision(con, "2-multi", 0, [8] * 3, [0.0, 0.01, 0.02], 1, [0.0, 1500.0, 3000.0])
    db.log_training_progress(con, "2-multi", "tabular", 50, -1700.5, 0.0)
    t = db.get_test_results(con)
    assert list(t.columns) == ["setting", "implementation", "agent", "day", "time", "load", "pv", "temperature",
                               "heatpump", "cost"]
    assert len(t) == 3 and t["heatpump"].tolist() == [0, 1500, 3000]
    r = db.get_rounds_decisions(con)
    assert r["round"].tolist() == [1, 1, 1] and r["decision"].tolist() == [0.0, 1500.0, 3000.0]
    assert len(db.get_validation_results(con)) == 2 and db.get_training_progress(con)["reward"][0] == -1700.5
