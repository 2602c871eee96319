"""open3d.pipelines counterpart (integration only — the reference uses nothing else from pipelines)."""
from . import integration  # noqa: F401
