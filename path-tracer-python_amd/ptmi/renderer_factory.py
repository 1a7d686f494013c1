"""String -> renderer registry (reference: src/render_server/renderer_factory.py:10-63).

'taichi' (the key every reference scene uses) and 'mi355x' both return the
MI355X renderer; the legacy pure-Python 'cpu'/'gpu' renderers are out of scope
 and raise like an unknown key.
"""
from .renderer import MI355XRenderer


class RendererFactory:
    _renderers = {'taichi': MI355XRenderer, 'mi355x': MI355XRenderer}

    @classmethod
    def create(cls, renderer_type, world, cam, img_path, **kwargs):
        key = renderer_type.lower()
        if key not in cls._renderers:
            raise ValueError(f"Unknown renderer type '{renderer_type}'. Available: {', '.join(cls._renderers)}")
        return cls._renderers[key](world, cam, img_path, **kwargs)

    @classmethod
    def get_available_renderers(cls):
        return list(cls._renderers)
