"""3-stage CPU graph: Frontend (HTTP /generate) -> Middle -> Backend (2 workers).

    python -m dynamo_exp_amd.sdk.serve hello_world:Frontend -f config.yaml --working-dir examples/hello_world
    curl -X POST localhost:8000/generate -d '{"text": "hi"}'
"""
import logging

from fastapi import FastAPI
from pydantic import BaseModel

from dynamo_exp_amd.sdk import ServiceConfig, depends, dynamo_endpoint, service

log = logging.getLogger(__name__)


class RequestType(BaseModel):
    text: str


@service(dynamo={"namespace": "inference"}, workers=2)
class Backend:
    def __init__(self):
        self.message = ServiceConfig.get_instance().get("Backend", {}).get("message", "back")

    @dynamo_endpoint()
    async def generate(self, req: RequestType):
        for token in f"{req.text}-{self.message}".split():
            yield f"Backend: {token}"


@service(dynamo={"namespace": "inference"})
class Middle:
    backend = depends(Backend)

    def __init__(self):
        self.message = ServiceConfig.get_instance().get("Middle", {}).get("message", "mid")

    @dynamo_endpoint()
    async def generate(self, req: RequestType):
        nxt = RequestType(text=f"{req.text}-{self.message}")
        async for r in self.backend.generate(nxt.model_dump_json()):
            yield f"Middle: {r}"


app = FastAPI(title="Hello World")


@service(dynamo={"namespace": "inference"}, app=app)
class Frontend:
    middle = depends(Middle)

    def __init__(self):
        self.message = ServiceConfig.get_instance().get("Frontend", {}).get("message", "front")

    @dynamo_endpoint(is_api=True)
    async def generate(self, request: RequestType):
        txt = RequestType(text=f"{request.text}-{self.message}")
        async for r in self.middle.generate(txt.model_dump_json()):
            yield f"Frontend: {r}"
