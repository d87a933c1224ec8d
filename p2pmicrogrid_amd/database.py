"""SQLite result sinks and data source with the reference's schema (mirrors microgrid/database.py).

The thesis's analysis scripts (data_analysis.py) read these tables, so a run of this package
can feed them directly:

    environment, load                   raw profiles (database.py:31-43), read by ``get_data``
    validation_results, test_results    per agent-step rows of a greedy day (database.py:59-71)
    rounds_comparison                   heat-pump decision of every negotiation round (:73-77)
    training_progress                   50-episode running means (log_training_progress :198-210;
                                        the reference never creates this table, create_tables
                                        here does)

Only the standard library's sqlite3 and pandas are used.  ``get_connection`` takes an explicit
path (the reference reads it from its absent, git-ignored ``config.py``).
"""
from __future__ import annotations

import os
import sqlite3
from datetime import datetime
from typing import List, Optional, Sequence, Union

import pandas as pd


def get_connection(path: Optional[str] = None) -> Optional[sqlite3.Connection]:
    """database.py:16-25; path defaults to $P2PMG_DB."""
    path = path or os.environ.get("P2PMG_DB")
    if not path:
        return None
    try:
        return sqlite3.connect(path)
    except sqlite3.Error as e:  # the reference prints and returns None
        print(e)
        return None


def create_tables(cursor: sqlite3.Cursor) -> None:
    """database.py:28-81 (same tables, keys and column order) + training_progress."""
    cursor.execute("""CREATE TABLE IF NOT EXISTS environment
        (date text NOT NULL, time text NOT NULL, utc text NOT NULL,
         temperature real, cloud_cover real, humidity real, irradiation real, pv real,
         PRIMARY KEY (date, time, utc))""")
    cursor.execute("""CREATE TABLE IF NOT EXISTS load
        (date text NOT NULL, time text NOT NULL, utc text NOT NULL, load_0 real,
         PRIMARY KEY (date, time, utc))""")
    cursor.execute("""CREATE TABLE IF NOT EXISTS validation_results
        (setting text NOT NULL, implementation text NOT NULL, agent integer NOT NULL, day integer NOT NULL,
         time real NOT NULL, load real, pv real, temperature real, heatpump real, cost real,
         PRIMARY KEY (setting, implementation, agent, day, time))""")
    cursor.execute("""CREATE TABLE IF NOT EXISTS test_results
        (setting text NOT NULL, implementation text NOT NULL, agent integer NOT NULL, day integer NOT NULL,
         time real NOT NULL, load real, pv real, temperature real, heatpump real, cost real,
         PRIMARY KEY (setting, implementation, agent, day, time))""")
    cursor.execute("""CREATE TABLE IF NOT EXISTS rounds_comparison
        (setting text NOT NULL, agent integer NOT NULL, day integer NOT NULL, time real NOT NULL,
         round integer NOT NULL, decision real,
         PRIMARY KEY (setting, agent, day, time, round))""")
    cursor.execute("""CREATE TABLE IF NOT EXISTS training_progress
        (setting text NOT NULL, implementation text NOT NULL, episode integer NOT NULL,
         reward real, error real)""")


def get_data(con: sqlite3.Connection, start: datetime, end: datetime) -> pd.DataFrame:
    """database.py:128-147: environment JOIN load over [start, end)."""
    q_env = "SELECT * FROM environment WHERE date >= ? AND date < ?"
    q_l = "SELECT * FROM load WHERE date >= ? AND date < ?"
    p = (start.strftime('%Y-%m-%d'), end.strftime('%Y-%m-%d'))
    df_env = pd.read_sql_query(q_env, con, params=p)
    df_l = pd.read_sql_query(q_l, con, params=p)
    return pd.merge(df_env, df_l, on=['date', 'time', 'utc'])


def _insert(con, query: str, records) -> None:
    if con is None:
        return
    cur = con.cursor()
    try:
        cur.executemany(query, records)
        con.commit()
    finally:
        cur.close()


def log_training_progress(con, setting: str, agent_type: str, episode: int, reward: float, error: float) -> None:
    """database.py:198-210"""
    _insert(con, "INSERT INTO training_progress VALUES (?,?,?,?,?)",
            [(setting, agent_type, int(episode), float(reward), float(error))])


def _results(setting, agent_id, days, time, load, pv, temperature, heatpump, cost, implementation):
    n = len(load)
    return [*zip([setting] * n, [implementation] * n, [int(agent_id)] * n, [int(d) for d in days],
                 [float(t) for t in time], [float(x) for x in load], [float(x) for x in pv],
                 [float(x) for x in temperature], [float(x) for x in heatpump], [float(x) for x in cost])]


def log_validation_results(con, setting: str, agent_id: int, days: Sequence[int], time: Sequence[float],
                           load, pv, temperature, heatpump, cost, implementation: str) -> None:
    """database.py:227-245"""
    _insert(con, "INSERT INTO validation_results VALUES (?,?,?,?,?,?,?,?,?,?)",
            _results(setting, agent_id, days, time, load, pv, temperature, heatpump, cost, implementation))


def log_test_results(con, setting: str, agent_id: int, days: Sequence[int], time: Sequence[float],
                     load, pv, temperature, heatpump, cost, implementation: str) -> None:
    """database.py:262-280"""
    _insert(con, "INSERT INTO test_results VALUES (?,?,?,?,?,?,?,?,?,?)",
            _results(setting, agent_id, days, time, load, pv, temperature, heatpump, cost, implementation))


def log_rounds_decision(con, setting: str, agent: int, days: Sequence[int], time: Sequence[float], round: int,
                        decisions: Sequence[float]) -> None:
    """database.py:296-312"""
    n = len(time)
    _insert(con, "INSERT INTO rounds_comparison VALUES (?,?,?,?,?,?)",
            [*zip([setting] * n, [int(agent)] * n, [int(d) for d in days], [float(t) for t in time],
                  [int(round)] * n, [float(x) for x in decisions])])


def _read(con, table: str) -> Union[pd.DataFrame, None]:
    return pd.read_sql_query(f"SELECT * FROM {table}", con) if con else None


def get_training_progress(con):
    return _read(con, "training_progress")


def get_validation_results(con):
    return _read(con, "validation_results")


def get_test_results(con):
    return _read(con, "test_results")


def get_rounds_decisions(con):
    return _read(con, "rounds_comparison")
