"""Drop-in for the reference's ``Utils/util.py`` (METR-LA path: loaders, scaler, adjacency,
masked metrics)."""
from gwn_amd.util import *  # noqa: F401,F403
from gwn_amd.util import (DataLoader, StandardScaler, asym_adj, load_adj, load_dataset, load_dataset_metr,  # noqa: F401
                          masked_mae, masked_mape, masked_mse, masked_rmse, metric, mod_adj, sym_adj)
