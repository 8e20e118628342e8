"""Lean serving SDK: `@service` graphs, `depends()`, `@dynamo_endpoint`,
YAML config, `serve` supervisor (reference deploy/dynamo/sdk, minus BentoML)."""
from .config import ServiceConfig
from .service import (DynamoClient, DynamoService, LeaseConfig, async_on_shutdown, async_on_start, depends,
                      dynamo_endpoint, service)

__all__ = ["service", "depends", "dynamo_endpoint", "async_on_start", "async_on_shutdown", "ServiceConfig",
           "DynamoService", "DynamoClient", "LeaseConfig"]
