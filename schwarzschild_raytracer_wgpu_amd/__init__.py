"""schwarzschild_raytracer_wgpu_amd — MI355X-native per-pixel Schwarzschild
geodesic renderer (drop-in for the sky-sphere path of
FirePrincess01/schwarzschild_raytracer_wgpu).  See DESIGN.md."""
from . import _lib  # noqa: F401  (raises if libgeo.so is missing: no CPU fallback)
from ._lib import GEO_MODE_ADAPTIVE, GEO_MODE_DIRECT, GEO_MODE_FAN, GeoError, GeoFrame, GeoScene  # noqa: F401
from ._lib import GEO_RAYS_FAR, GEO_RAYS_NEAR  # noqa: F401
from .api import (BasicSphereBuffer, Context, Observer, PointCloud, RayConnectors, Renderer,  # noqa: F401
                  RenderTarget, SphereRayTracer, draw_points, make_scene)
