"""Tiered HBM/host/disk cache + CDC invalidation (reference crates/cache, crates/cdc)."""
from .cdc import CachedTable, CdcManager, ChangeEvent
from .tiered import Cache, CacheConfig, InMemoryCache, TieredCache

__all__ = ["Cache", "CacheConfig", "InMemoryCache", "TieredCache", "CdcManager", "ChangeEvent", "CachedTable"]
