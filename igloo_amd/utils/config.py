"""One configuration object: file (JSON / YAML / TOML) < ``IGLOO_*`` env < CLI flags.

The reference accepts ``--config`` but ignores it (reference
crates/igloo/src/main.rs:36-39) and hard-codes ports 50051/50052, the 5 s
heartbeat, channel capacities and batch sizes. All of those are
settings here.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, fields
from typing import Any, Dict, Optional


@dataclass
class IglooConfig:
    # service endpoints (reference defaults: coordinator 127.0.0.1:50051, worker 127.0.0.1:50052)
    coordinator_host: str = "127.0.0.1"
    coordinator_port: int = 50051
    worker_host: str = "127.0.0.1"
    worker_port: int = 50052
    # liveness (reference worker heartbeats every 5 s, coordinator never evicts)
    heartbeat_interval_s: float = 5.0
    heartbeat_timeout_s: float = 15.0
    # upper bound of any data collective inside a worker group (then the group is broken)
    collective_timeout_s: float = 60.0
    # after a supervised worker group fails, wait this long for the node
    # supervisor's replacement group on the surviving GPUs (service/supervisor.py)
    recovery_wait_s: float = 30.0
    # execution
    device: Optional[str] = None
    gpus_per_node: int = 8
    broadcast_rows: int = 4_000_000
    # cache tiers (HBM / host / disk)
    cache_hbm_gb: float = 64.0
    cache_host_gb: float = 32.0
    cache_dir: Optional[str] = None
    # tables: name -> {"format": parquet|csv|iceberg|postgres|mysql, "path"/"dsn": ..., ...}
    tables: Dict[str, Dict[str, Any]] = field(default_factory=dict)
    auth_token: Optional[str] = None
    log_level: str = "warning"
    fault: Optional[str] = None   # fault-injection spec (utils/faults.py), e.g. "drop_heartbeat"

    def to_dict(self) -> dict:
        return asdict(self)


def _parse_file(path: str) -> dict:
    with open(path, "rb") as f:
        raw = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        return yaml.safe_load(raw) or {}
    if path.endswith(".toml"):
        try:
            import tomllib  # type: ignore
        except ImportError:
            import tomli as tomllib  # type: ignore
        return tomllib.loads(raw.decode())
    return json.loads(raw.decode() or "{}")


def load_config(path: Optional[str] = None, overrides: Optional[dict] = None) -> IglooConfig:
    data: Dict[str, Any] = {}
    if path:
        data.update(_parse_file(path))
    names = {f.name: f for f in fields(IglooConfig)}
    for k, f in names.items():
        env = os.environ.get("IGLOO_" + k.upper())
        if env is not None:
            if f.type in ("int", int):
                data[k] = int(env)
            elif f.type in ("float", float):
                data[k] = float(env)
            else:
                data[k] = env
    for k, v in (overrides or {}).items():
        if v is not None:
            data[k] = v
    unknown = set(data) - set(names)
    if unknown:
        raise ValueError(f"unknown config keys: {sorted(unknown)}")
    return IglooConfig(**data)


def register_config_tables(engine, cfg: IglooConfig):
    for name, spec in cfg.tables.items():
        fmt = spec.get("format", "parquet").lower()
        if fmt == "parquet":
            engine.register_parquet(name, spec["path"])
        elif fmt == "csv":
            engine.register_csv(name, spec["path"], has_header=spec.get("header", True),
                                delimiter=spec.get("delimiter", ","))
        elif fmt == "iceberg":
            engine.register_iceberg(name, spec["path"])
        elif fmt == "postgres":
            from ..connectors.postgres import PostgresTable
            engine.register_table(name, PostgresTable(spec["dsn"], spec.get("table", name), query=spec.get("query"),
                                                      version_sql=spec.get("version_sql")))
        elif fmt == "mysql":
            from ..connectors.mysql import MySqlTable
            engine.register_table(name, MySqlTable(spec["dsn"], spec.get("table", name), query=spec.get("query"),
                                                   version_sql=spec.get("version_sql")))
        else:
            raise ValueError(f"unknown table format {fmt}")
