"""Extract the renderer's golden frames from the reference's demo GIFs
(readme.md:64: demo/navigation/3agents.gif and 24agents.gif, frame 0) as
lossless PNGs.
Run where /root/reference exists: python tests/golden/make_render_fixture.py
The GIF is read with Pillow (an image decoder; nothing in it is executed)."""
from pathlib import Path

from PIL import Image

SRC = Path("/root/reference/demo/navigation")
HERE = Path(__file__).resolve().parent

if __name__ == "__main__":
    for n in (3, 24):
        im = Image.open(SRC / f"{n}agents.gif")
        im.seek(0)
        out = HERE / f"demo_nav{n}_f0.png"
        im.convert("RGB").save(out, optimize=True)
        print(out, out.stat().st_size, "bytes")
