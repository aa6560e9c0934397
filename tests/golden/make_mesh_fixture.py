"""Convert the reference's own mesh fixture (mesh_loading/x1.2562.grid.nc, netCDF CDF-2)
and its partition file (x1.2562.graph.info.part.16) into compact numpy fixtures that
travel with the repo (the GPU box has no /root/reference).

Data only: every array is copied verbatim from the netCDF variables the reference
reads in mesh_loading.rg:123-201 (ids stay 1-based, distances stay on the unit sphere).
Run in the build container:  python tests/golden/make_mesh_fixture.py
"""
import os
import numpy as np
from scipy.io import netcdf_file

REF = "/root/reference/mesh_loading"
OUT = os.path.dirname(os.path.abspath(__file__))

VARS = ["latCell", "lonCell", "xCell", "yCell", "zCell", "meshDensity", "areaCell",
        "nEdgesOnCell", "edgesOnCell", "cellsOnCell", "verticesOnCell",
        "latEdge", "lonEdge", "xEdge", "yEdge", "zEdge", "cellsOnEdge", "verticesOnEdge",
        "nEdgesOnEdge", "edgesOnEdge", "weightsOnEdge", "dvEdge", "dcEdge", "angleEdge",
        "latVertex", "lonVertex", "xVertex", "yVertex", "zVertex", "areaTriangle",
        "edgesOnVertex", "cellsOnVertex", "kiteAreasOnVertex"]


def main():
    f = netcdf_file(os.path.join(REF, "x1.2562.grid.nc"), "r", mmap=False)
    out = {}
    for v in VARS:
        a = np.asarray(f.variables[v].data)
        out[v] = a.astype(np.int32 if a.dtype.kind == "i" else np.float64)
    part = np.loadtxt(os.path.join(REF, "x1.2562.graph.info.part.16"), dtype=np.int32)
    out["graph_info_part_16"] = part
    np.savez_compressed(os.path.join(OUT, "x1.2562.mesh.npz"), **out)
    print("wrote", os.path.join(OUT, "x1.2562.mesh.npz"), {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
