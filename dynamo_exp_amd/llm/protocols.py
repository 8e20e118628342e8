"""Wire protocols: OpenAI-compatible API types (+ `nvext`) and the internal
token-level protocol between the frontend/preprocessor and engines.

Field names follow the reference so payloads are interchangeable:
  * NvExt                 lib/llm/src/protocols/openai/nvext.rs:28
  * StopConditions        lib/llm/src/protocols/common.rs:205
  * SamplingOptions       lib/llm/src/protocols/common.rs:248
  * PreprocessedRequest   lib/llm/src/protocols/common/preprocessor.rs:25
  * LLMEngineOutput       lib/llm/src/protocols/common/llm_backend.rs:60
"""
from __future__ import annotations

import time
import uuid
from typing import Any, Literal, Optional, Union

from pydantic import BaseModel, ConfigDict, Field


class NvExt(BaseModel):
    model_config = ConfigDict(extra="allow")
    ignore_eos: Optional[bool] = None
    top_k: Optional[int] = None
    repetition_penalty: Optional[float] = None
    greed_sampling: Optional[bool] = None
    use_raw_prompt: Optional[bool] = None
    annotations: Optional[list[str]] = None


class ChatMessage(BaseModel):
    model_config = ConfigDict(extra="allow")
    role: str
    content: Optional[Union[str, list[dict[str, Any]]]] = None
    name: Optional[str] = None
    tool_calls: Optional[list[dict[str, Any]]] = None
    tool_call_id: Optional[str] = None

    def text(self) -> str:
        if isinstance(self.content, str) or self.content is None:
            return self.content or ""
        return "".join(p.get("text", "") for p in self.content if isinstance(p, dict))


class StreamOptions(BaseModel):
    include_usage: Optional[bool] = None


class _SamplingFields(BaseModel):
    model_config = ConfigDict(extra="allow")
    model: str
    max_tokens: Optional[int] = None
    max_completion_tokens: Optional[int] = None
    min_tokens: Optional[int] = None
    temperature: Optional[float] = None
    top_p: Optional[float] = None
    top_k: Optional[int] = None
    min_p: Optional[float] = None
    n: Optional[int] = None
    stream: Optional[bool] = False
    stream_options: Optional[StreamOptions] = None
    stop: Optional[Union[str, list[str]]] = None
    seed: Optional[int] = None
    presence_penalty: Optional[float] = None
    frequency_penalty: Optional[float] = None
    repetition_penalty: Optional[float] = None
    logprobs: Optional[Union[bool, int]] = None
    top_logprobs: Optional[int] = None
    user: Optional[str] = None
    ignore_eos: Optional[bool] = None
    nvext: Optional[NvExt] = None

    def stop_list(self) -> list[str]:
        if self.stop is None:
            return []
        return [self.stop] if isinstance(self.stop, str) else list(self.stop)


class ChatCompletionRequest(_SamplingFields):
    messages: list[ChatMessage]
    tools: Optional[list[dict[str, Any]]] = None
    tool_choice: Optional[Any] = None
    chat_template_kwargs: Optional[dict[str, Any]] = None


class CompletionRequest(_SamplingFields):
    prompt: Union[str, list[str], list[int], list[list[int]]]
    echo: Optional[bool] = None
    suffix: Optional[str] = None


# ---------------------------------------------------------------- responses
class Usage(BaseModel):
    prompt_tokens: int = 0
    completion_tokens: int = 0
    total_tokens: int = 0


class ChatDelta(BaseModel):
    role: Optional[str] = None
    content: Optional[str] = None
    tool_calls: Optional[list[dict]] = None


class ChatChunkChoice(BaseModel):
    index: int = 0
    delta: ChatDelta
    finish_reason: Optional[str] = None
    logprobs: Optional[dict] = None


class ChatCompletionChunk(BaseModel):
    id: str
    object: Literal["chat.completion.chunk"] = "chat.completion.chunk"
    created: int = Field(default_factory=lambda: int(time.time()))
    model: str
    choices: list[ChatChunkChoice]
    usage: Optional[Usage] = None
    system_fingerprint: Optional[str] = None


class ChatChoice(BaseModel):
    index: int = 0
    message: ChatMessage
    finish_reason: Optional[str] = None
    logprobs: Optional[dict] = None


class ChatCompletionResponse(BaseModel):
    id: str
    object: Literal["chat.completion"] = "chat.completion"
    created: int = Field(default_factory=lambda: int(time.time()))
    model: str
    choices: list[ChatChoice]
    usage: Optional[Usage] = None


class CompletionChoice(BaseModel):
    index: int = 0
    text: str = ""
    finish_reason: Optional[str] = None
    logprobs: Optional[dict] = None


class CompletionResponse(BaseModel):
    id: str
    object: Literal["text_completion"] = "text_completion"
    created: int = Field(default_factory=lambda: int(time.time()))
    model: str
    choices: list[CompletionChoice]
    usage: Optional[Usage] = None


class ModelInfo(BaseModel):
    id: str
    object: str = "model"
    created: int = Field(default_factory=lambda: int(time.time()))
    owned_by: str = "dynamo_exp_amd"


class ModelList(BaseModel):
    object: str = "list"
    data: list[ModelInfo]


# ---------------------------------------------------------------- internal (token level)
class StopConditions(BaseModel):
    max_tokens: Optional[int] = None
    stop: Optional[list[str]] = None
    stop_token_ids_hidden: Optional[list[int]] = None
    min_tokens: Optional[int] = None
    ignore_eos: Optional[bool] = None

    def apply_ignore_eos(self) -> None:
        """reference common.rs:216 -- ignore_eos implies min_tokens = max_tokens."""
        if self.ignore_eos and self.max_tokens is not None:
            self.min_tokens = self.max_tokens


class SamplingOptions(BaseModel):
    n: Optional[int] = None
    best_of: Optional[int] = None
    presence_penalty: Optional[float] = None
    frequency_penalty: Optional[float] = None
    repetition_penalty: Optional[float] = None
    temperature: Optional[float] = None
    top_p: Optional[float] = None
    top_k: Optional[int] = None
    min_p: Optional[float] = None
    use_beam_search: Optional[bool] = None
    length_penalty: Optional[float] = None
    seed: Optional[int] = None
    greed_sampling: Optional[bool] = None


class OutputOptions(BaseModel):
    logprobs: Optional[int] = None
    prompt_logprobs: Optional[int] = None
    skip_special_tokens: Optional[bool] = None
    formatted_prompt: Optional[bool] = None


class PreprocessedRequest(BaseModel):
    model_config = ConfigDict(extra="allow")
    token_ids: list[int]
    stop_conditions: StopConditions = Field(default_factory=StopConditions)
    sampling_options: SamplingOptions = Field(default_factory=SamplingOptions)
    output_options: OutputOptions = Field(default_factory=OutputOptions)
    eos_token_ids: list[int] = Field(default_factory=list)
    mdc_sum: Optional[str] = None
    annotations: list[str] = Field(default_factory=list)
    # routing / disaggregation hints
    estimated_prefix_hit_num_blocks: Optional[int] = None
    request_id: Optional[str] = None
    # multimodal inputs: {"image_urls": [...]} (placeholders already expanded in token_ids)
    multi_modal: Optional[dict[str, Any]] = None


class LLMEngineOutput(BaseModel):
    token_ids: list[int] = Field(default_factory=list)
    tokens: Optional[list[str]] = None
    text: Optional[str] = None
    cum_log_probs: Optional[float] = None
    log_probs: Optional[list[float]] = None
    finish_reason: Optional[str] = None


class Annotated(BaseModel):
    """Stream item wrapper {data, id, event, comment} (protocols/annotated.rs:32)."""

    data: Optional[Any] = None
    id: Optional[str] = None
    event: Optional[str] = None
    comment: Optional[list[str]] = None

    @classmethod
    def error(cls, msg: str) -> "Annotated":
        return cls(event="error", comment=[msg])


def new_request_id(prefix: str = "chatcmpl") -> str:
    return f"{prefix}-{uuid.uuid4().hex}"


FINISH_MAP = {"stop": "stop", "length": "length", "cancelled": "stop", "error": "error", "eos": "stop",
              "remote_decode": "stop"}
