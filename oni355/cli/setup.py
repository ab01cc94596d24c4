"""``oni-setup`` -- lay down a deployment: storage layout, table schemas and config templates.

The reference's oni-setup module ([U-M]) ran ``hdfs_setup.sh``:
HDFS folders ``${HUSER}/{flow,dns,proxy}/{hive,stage,...}``, Hive DDL creating the external
Parquet tables partitioned by y/m/d/h, and a ``duxbay.conf`` template for the ML/OA nodes. Here
the store is the local columnar day store (``oni355.store.columnar``), so setup creates

  <DATA_ROOT>/<source>/            day partitions land here (``<YYYYMMDD>/[part-NNNNN/]<col>.npy``)
  <DATA_ROOT>/<source>/_table.json the table definition (the DDL's role): column order + kinds
  <LPATH>/<source>/                ML results / OA scores / feedback files
  <STAGE>/<source>/                collector drop directory (ingest staging)
  <CONF_DIR>/duxbay.conf           KEY=VALUE template of every oni355.config key (parsed, never sourced)
  <CONF_DIR>/ingest_conf.json      the reference ingest_conf.json layout, pointing at the folders above

  oni-setup --data-root ./oni_store --lpath ./oni_data --stage ./oni_stage --conf-dir ./conf [--force]

Idempotent: existing folders are kept; templates are only rewritten with ``--force``.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys

from .. import schema
from ..config import OniConfig

# column kinds as the ingest decoders store them (strings: offsets + chars, see columnar.py)
_STRING_COLUMNS = {
    "flow": {"treceived"},
    "dns": {"frame_time", "dns_qry_name", "dns_a"},
    "proxy": {"p_date", "p_time", "host", "reqmethod", "useragent", "resconttype", "username", "authgroup",
              "exceptionid", "filterresult", "webcat", "referer", "action", "urischeme", "uripath", "uriquery",
              "uriextension", "virusid", "bcappname", "bcappoperation", "fulluri"},
}
_IP_COLUMNS = {"sip", "dip", "rip", "ip_src", "ip_dst", "clientip", "serverip"}
_FLOAT_COLUMNS = {"tdur", "duration"}
_INT64_COLUMNS = {"unix_tstamp", "ipkt", "ibyt", "opkt", "obyt", "scbytes", "csbytes"}


def table_definition(source: str) -> dict:
    """Column order + storage kind of a source's raw table (the reference's Hive DDL role)."""
    cols = []
    for c in schema.raw_columns(source):
        if c in _STRING_COLUMNS[source]:
            kind = "string"
        elif c in _IP_COLUMNS:
            kind = "uint32"  # IPv4 as integer
        elif c in _FLOAT_COLUMNS:
            kind = "float64"
        elif c in _INT64_COLUMNS:
            kind = "int64"
        else:
            kind = "int32"
        cols.append({"name": c, "kind": kind})
    return {"source": source, "partitioning": "<YYYYMMDD>/[part-NNNNN/]", "columns": cols,
            "results_columns": schema.result_columns(source), "scores_columns": schema.score_columns(source)}


def duxbay_template(cfg: OniConfig) -> str:
    lines = ["# oni355 configuration (duxbay.conf layout: KEY=VALUE, parsed -- never sourced)",
             "# precedence: built-in defaults < this file < ONI_<KEY> environment < CLI flags"]
    for f in dataclasses.fields(OniConfig):
        if f.name == "extra":
            continue
        v = getattr(cfg, f.name)
        lines.append(f"{f.name}={json.dumps(v) if isinstance(v, str) else v}")
    return "\n".join(lines) + "\n"


def ingest_template(data_root: str, stage: str) -> dict:
    files = {"flow": "nfcapd.*", "dns": "*.pcap", "proxy": "*.log"}
    return {
        "dbname": "oni", "data_root": os.path.abspath(data_root),
        "pipelines": {src: {"type": src, "collector_path": os.path.abspath(os.path.join(stage, src)),
                            "local_staging": os.path.abspath(os.path.join(stage, src, ".work")),
                            "supported_files": [files[src]], "process_opt": ""}
                      for src in schema.SOURCES},
    }


def _write(path: str, text: str, force: bool) -> bool:
    if os.path.exists(path) and not force:
        return False
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)
    return True


def setup(data_root: str, lpath: str, stage: str, conf_dir: str, force: bool = False) -> dict:
    made, written = [], []
    for src in schema.SOURCES:
        for d in (os.path.join(data_root, src), os.path.join(lpath, src), os.path.join(stage, src),
                  os.path.join(stage, src, ".work")):
            if not os.path.isdir(d):
                os.makedirs(d, exist_ok=True)
                made.append(d)
        if _write(os.path.join(data_root, src, "_table.json"), json.dumps(table_definition(src), indent=1), force):
            written.append(os.path.join(data_root, src, "_table.json"))
    os.makedirs(conf_dir, exist_ok=True)
    cfg = OniConfig().replace(DATA_ROOT=os.path.abspath(data_root), LPATH=os.path.abspath(lpath))
    if _write(os.path.join(conf_dir, "duxbay.conf"), duxbay_template(cfg), force):
        written.append(os.path.join(conf_dir, "duxbay.conf"))
    if _write(os.path.join(conf_dir, "ingest_conf.json"), json.dumps(ingest_template(data_root, stage), indent=1),
              force):
        written.append(os.path.join(conf_dir, "ingest_conf.json"))
    return {"created_dirs": made, "written": written}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="oni-setup", description=__doc__.split("\n")[0])
    ap.add_argument("--data-root", default=os.environ.get("ONI_DATA_ROOT", "./oni_store"))
    ap.add_argument("--lpath", default=os.environ.get("ONI_LPATH", "./oni_data"))
    ap.add_argument("--stage", default="./oni_stage")
    ap.add_argument("--conf-dir", default="./conf")
    ap.add_argument("--force", action="store_true", help="rewrite existing table definitions / templates")
    a = ap.parse_args(argv)
    print(json.dumps(setup(a.data_root, a.lpath, a.stage, a.conf_dir, a.force)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
