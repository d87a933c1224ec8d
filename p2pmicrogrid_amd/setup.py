"""Parameters for creating, training and running a community (mirrors microgrid/setup.py:1-36).

Same module-level names as the reference so ``import setup``-style callers keep working:
``from p2pmicrogrid_amd import setup``.
"""
from datetime import datetime

# Constants (setup.py:8-13)
SECONDS_PER_MINUTE = 60
MINUTES_PER_HOUR = 60
SECONDS_PER_HOUR = SECONDS_PER_MINUTE * MINUTES_PER_HOUR
HOURS_PER_DAY = 24
CENTS_PER_EURO = 100
KWH_TO_WS = 1 * 1e3 * SECONDS_PER_HOUR

# Simulation settings (setup.py:15-26)
TIME_SLOT = 15
HORIZON = 24
START = datetime(2021, 11, 1)
END = datetime(2021, 11, 2)
DURATION = (END - START).total_seconds() / SECONDS_PER_MINUTE / TIME_SLOT
GRID_COST_AVG = 12.0        # c€ / kWh
GRID_COST_AMPLITUDE = 5.0   # c€ / kWh
GRID_COST_PERIOD = 12
GRID_COST_PHASE = 3
GRID_INJECTION_PRICE = 0.07     # € / kWh
seed = 42

# Community parameters (setup.py:28-36)
starting_episodes = 0
max_episodes = 1000
min_episodes_criterion = 50
save_episodes = 50
nr_agents = 2
rounds = 1
homogeneous = False
implementation = 'tabular'      # Agent implementation

# Build-specific knobs (not in the reference)
q_dtype = 'f64'    # 'f64' = the reference's float64 table (bit-exact); 'f32' = throughput mode
device = 0         # HIP device of the single-community (drop-in) path
