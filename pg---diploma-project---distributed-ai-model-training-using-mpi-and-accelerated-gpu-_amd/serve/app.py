"""Web inference demo (reference: the Gradio app printed in GROUP03.pdf p.26-27).

Reference behaviour: load ``best_mobilenetv2_cifar10_224.pth`` into a
MobileNetV2 with a 10-class head, ``predict(img) -> {class: prob}`` for the
top 3, ``gr.Interface(fn=predict, inputs=gr.Image(type="pil"),
outputs=gr.Label(num_top_classes=3), title="CIFAR-10 MobileNetV2 Classifier")``,
``launch(server_name="0.0.0.0", server_port=7861)``.

* If ``gradio`` is importable the same Interface is built.
* Otherwise (it is not installed in this environment) an equivalent FastAPI app
  is served on the same host/port: ``POST /predict`` with the raw image bytes
  returns ``{"label": {class: prob}}`` (top-3), ``GET /`` a minimal upload page.

Normalisation defaults to the training statistics (ImageNet); ``--normalize
cifar`` reproduces the reference app's mismatched CIFAR constants.

  python -m pgdist.serve.app --checkpoint best_mobilenetv2_cifar10_224.pth
"""
import argparse
import io

from .predict import Predictor

TITLE = "CIFAR-10 MobileNetV2 Classifier"

_PAGE = """<!doctype html><html><head><title>{title}</title></head><body>
<h2>{title}</h2><p>Upload CIFAR-10 style image</p>
<input type=file id=f accept="image/*"><pre id=o></pre>
<script>
document.getElementById('f').onchange = async (e) => {{
  const r = await fetch('/predict', {{method: 'POST', body: e.target.files[0]}});
  document.getElementById('o').textContent = JSON.stringify(await r.json(), null, 2);
}};
</script></body></html>"""


def build_gradio(predictor: Predictor):
    import gradio as gr

    def predict(img):
        return predictor.label_dict(img, 3)

    return gr.Interface(fn=predict, inputs=gr.Image(type="pil", label="Upload CIFAR-10 style image"),
                        outputs=gr.Label(num_top_classes=3, label="Top-3 predictions"), title=TITLE)


def build_fastapi(predictor: Predictor):
    from fastapi import FastAPI, Request
    from fastapi.responses import HTMLResponse, JSONResponse

    app = FastAPI(title=TITLE)

    @app.get("/", response_class=HTMLResponse)
    def index():
        return _PAGE.format(title=TITLE)

    @app.post("/predict")
    async def predict(request: Request):
        data = await request.body()
        if not data:
            return JSONResponse({"error": "empty body: POST the image bytes"}, status_code=400)
        return {"label": predictor.label_dict(io.BytesIO(data), 3)}

    @app.get("/healthz")
    def healthz():
        return {"ok": True, "device": str(predictor.device)}

    return app


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--checkpoint", default="best_mobilenetv2_cifar10_224.pth")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=7861)
    ap.add_argument("--normalize", choices=("imagenet", "cifar"), default="imagenet")
    ap.add_argument("--device", default="auto")
    ap.add_argument("--model", default="mobilenet_v2", help="mobilenet_v2 | resnet50 (checkpoint architecture)")
    a = ap.parse_args(argv)
    pred = Predictor(a.checkpoint, device=a.device, normalize=a.normalize, model_name=a.model)
    try:
        demo = build_gradio(pred)
        demo.launch(server_name=a.host, server_port=a.port)
    except ImportError:
        import uvicorn
        uvicorn.run(build_fastapi(pred), host=a.host, port=a.port)


if __name__ == "__main__":
    main()
