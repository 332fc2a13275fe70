"""Environment plugins shipped with handyrl_amd (same API as handyrl.envs)."""
