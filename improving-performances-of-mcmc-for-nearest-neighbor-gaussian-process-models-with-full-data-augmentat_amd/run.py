"""mcmc_nngp_run -- host mirror of Scripts/mcmc_nngp_run.R:1-52 (cycle driver,
records merge, Gelman-Rubin-Brooks stop).  Plots are out of scope."""
from __future__ import annotations

import time

import numpy as np

from .diagnose import ESS, Gelman_Rubin_Brooks
from .update_gaussian import mcmc_nngp_update_Gaussian


def mcmc_nngp_run(mcmc_nngp_list, Gelman_Rubin_Brooks_stop=(1.1, 1.1), burn_in=0.5, n_cores=None,
                  field_thinning=1.0, n_iterations_update=200, ancillary=True, n_chromatic=10,
                  save_name=None, n_cycles=1, plot_beta=False, verbose=True, on_chol_error="error"):
    L = mcmc_nngp_list
    cycle = 1
    while cycle <= n_cycles:
        if verbose:
            print(f"cycle = {cycle}")
        if L["space_time_model"]["response_model"] != "Gaussian":
            raise NotImplementedError("only the Gaussian response model exists in the reference (run.R:12)")
        first = next(iter(L["records"].values()))
        res = mcmc_nngp_update_Gaussian(
            locs=L["locs"], X=L["X"], observed_field=L["observed_field"],
            space_time_model=L["space_time_model"], vecchia_approx=L["vecchia_approx"],
            states=L["states"], iterations=first["iterations"],  # chain 1's matrix for all (run.R:16)
            n_iterations_update=n_iterations_update, n_cores=n_cores, field_thinning=field_thinning,
            ancillary=ancillary, n_chromatic=n_chromatic, contexts=L.get("_contexts"), seed=L.get("seed", 1),
            on_chol_error=on_chol_error)
        for name, rec in L["records"].items():
            L["states"][name] = res[name]["state"]
            iter_start = rec["iterations"][-1, 0]
            its = np.arange(1, n_iterations_update + 1)
            saved = its[np.round(its * field_thinning) == its * field_thinning]
            rec["saved_field"] = np.concatenate([rec.get("saved_field", np.zeros(0)), iter_start + saved])
            rec["iterations"] = np.vstack([rec["iterations"],
                                           [iter_start + n_iterations_update, time.time() - L["t_begin"]]])
            for k, v in res[name]["records"].items():
                old = rec["params"].get(k)
                rec["params"][k] = v if old is None else np.vstack([old, v])
        grb = Gelman_Rubin_Brooks(L["records"], burn_in)
        L["diagnostics"]["Gelman_Rubin_Brooks"].append(grb)
        L["diagnostics"].setdefault("ESS", []).append(ESS(L["records"], burn_in))
        if verbose:
            print("Gelman-Rubin-Brooks R-hat : ")
            print(dict(zip(grb["names"], np.round(grb["R_hat"], 4))))
        rh = grb["R_hat"]
        if rh[0] < Gelman_Rubin_Brooks_stop[0] or np.all(rh[1:] < Gelman_Rubin_Brooks_stop[1]):
            break
        cycle += 1
    return L
