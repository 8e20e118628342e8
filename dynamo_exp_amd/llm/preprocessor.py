"""OpenAI preprocessor: chat template + tokenization on the way in, OpenAI
stream chunks on the way out (reference lib/llm/src/preprocessor.rs:63-330).

* chat template: the model's `tokenizer_config.json` jinja `chat_template`
  (HF semantics: messages, tools, add_generation_prompt, bos/eos tokens,
  raise_exception, strftime_now) or a built-in Llama-3 template; the
  `llama3_date_time` context mixin provides `date_string`;
* hidden stop ids = request stop ids + model EOS (unless ignore_eos);
* annotations: `formatted_prompt` and `token_ids` are echoed back as stream
  events when requested via nvext.annotations.
"""
from __future__ import annotations

import datetime
import time
from typing import Any, AsyncIterator, Callable

import jinja2

from ..runtime.context import Context
from .protocols import (
    FINISH_MAP,
    ChatChoice,
    ChatCompletionChunk,
    ChatCompletionRequest,
    ChatCompletionResponse,
    ChatMessage,
    CompletionChoice,
    CompletionRequest,
    CompletionResponse,
    OutputOptions,
    PreprocessedRequest,
    SamplingOptions,
    StopConditions,
    Usage,
    new_request_id,
)
from .tokenizer import Tokenizer

LLAMA3_TEMPLATE = (
    "{{ bos_token }}"
    "{% for message in messages %}"
    "{{ '<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n' + (message['content'] | string | trim) + '<|eot_id|>' }}"
    "{% endfor %}"
    "{% if add_generation_prompt %}{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}{% endif %}"
)

# Llama 3.1 instruct prompt format (system header with knowledge / today
# dates, custom tools as JSON in the first user turn), written to reproduce
# the reference's formatted-prompt snapshots
# (lib/llm/tests/snapshots/preprocessor__*@meta_llama_llama_3_1_70b_instruct*.snap,
# tests/test_parity_fixtures.py).  Used with the "llama3_date_time" mixin.
LLAMA31_TEMPLATE = (
    "{%- if date_string is not defined %}{% set date_string = '26 Jul 2024' %}{% endif -%}"
    "{%- if messages and messages[0]['role'] == 'system' -%}"
    "{%- set system_message = messages[0]['content'] | trim %}{% set loop_messages = messages[1:] -%}"
    "{%- else -%}{%- set system_message = '' %}{% set loop_messages = messages -%}{%- endif -%}"
    "{{- bos_token + '<|start_header_id|>system<|end_header_id|>\n\n' -}}"
    "{%- if tools %}{{- 'Environment: ipython\n' -}}{% endif -%}"
    "{{- 'Cutting Knowledge Date: December 2023\nToday Date: ' + date_string + '\n\n' -}}"
    "{{- system_message + '<|eot_id|>' -}}"
    "{%- set ns = namespace(tools_done=false) -%}"
    "{%- for message in loop_messages -%}"
    "{{- '<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n' -}}"
    "{%- if tools and message['role'] == 'user' and not ns.tools_done -%}"
    "{{- 'Given the following functions, please respond with a JSON for a function call with its proper "
    "arguments that best answers the given prompt.\n\n' -}}"
    "{{- 'Respond in the format {\"name\": function name, \"parameters\": dictionary of argument name and its "
    "value}.Do not use variables.\n\n' -}}"
    "{%- for t in tools %}{{- t | tojson(indent=4) + '\n\n' -}}{% endfor -%}"
    "{%- set ns.tools_done = true -%}"
    "{%- endif -%}"
    "{{- (message['content'] or '') | trim + '<|eot_id|>' -}}"
    "{%- endfor -%}"
    "{%- if add_generation_prompt %}{{- '<|start_header_id|>assistant<|end_header_id|>\n\n' -}}{% endif -%}"
)


def _tojson(v, indent=None) -> str:
    """Jinja `tojson` as the reference's template engine (minijinja) renders
    it: keys sorted, HTML-sensitive characters escaped as \\uXXXX."""
    import json

    out = json.dumps(v, indent=indent, sort_keys=True, ensure_ascii=False)
    for ch, esc in (("&", "\\u0026"), ("'", "\\u0027"), ("<", "\\u003c"), (">", "\\u003e")):
        out = out.replace(ch, esc)
    return out


ANNOTATION_FORMATTED_PROMPT = "formatted_prompt"
IMAGE_MARKER = "<image>"
ANNOTATION_TOKEN_IDS = "token_ids"


class PromptFormatter:
    def __init__(self, template: str | None, bos_token: str = "", eos_token: str = "", mixins: list[str] | None = None):
        env = jinja2.Environment(trim_blocks=True, lstrip_blocks=True, undefined=jinja2.ChainableUndefined)

        def raise_exception(msg):
            raise jinja2.TemplateError(msg)

        env.globals["raise_exception"] = raise_exception
        env.globals["strftime_now"] = lambda fmt: datetime.datetime.now().strftime(fmt)
        env.filters["tojson"] = _tojson
        self.template = env.from_string(template or LLAMA3_TEMPLATE)
        self.bos, self.eos = bos_token, eos_token
        self.mixins = mixins or []

    def render(self, messages: list[dict], tools: list | None = None, add_generation_prompt: bool = True,
               **kwargs) -> str:
        ctx = dict(messages=messages, tools=tools, add_generation_prompt=add_generation_prompt,
                   bos_token=self.bos, eos_token=self.eos, **kwargs)
        if "llama3_date_time" in self.mixins:
            ctx.setdefault("date_string", datetime.date.today().strftime("%d %b %Y"))
        return self.template.render(**ctx)


class OpenAIPreprocessor:
    def __init__(self, model_name: str, tokenizer: Tokenizer, formatter: PromptFormatter | None = None,
                 eos_token_ids: list[int] | None = None, mdc_sum: str | None = None, context_length: int = 8192):
        self.model_name = model_name
        self.tok = tokenizer
        self.formatter = formatter or PromptFormatter(None, tokenizer.bos_token, tokenizer.eos_token)
        self.eos = list(eos_token_ids if eos_token_ids is not None else tokenizer.eos_token_ids)
        self.mdc_sum = mdc_sum
        self.context_length = context_length
        # multimodal (LLaVA): image parts become `image_tokens` placeholder ids
        self.image_token_id: int | None = None
        self.image_tokens = 0

    # ------------------------------------------------------------------ in
    def _common(self, req, token_ids: list[int]) -> PreprocessedRequest:
        nv = req.nvext
        ignore_eos = bool(req.ignore_eos or (nv and nv.ignore_eos))
        max_tokens = req.max_completion_tokens or req.max_tokens
        if max_tokens is None:
            max_tokens = max(1, self.context_length - len(token_ids))
        sc = StopConditions(max_tokens=max_tokens, stop=req.stop_list() or None, stop_token_ids_hidden=None,
                            min_tokens=req.min_tokens, ignore_eos=ignore_eos)
        top_k = req.top_k if req.top_k is not None else (nv.top_k if nv else None)
        so = SamplingOptions(
            n=req.n, presence_penalty=req.presence_penalty, frequency_penalty=req.frequency_penalty,
            repetition_penalty=req.repetition_penalty if req.repetition_penalty is not None else
            (nv.repetition_penalty if nv else None),
            temperature=req.temperature, top_p=req.top_p, top_k=top_k if (top_k or 0) > 0 else None, min_p=req.min_p,
            seed=req.seed, greed_sampling=(nv.greed_sampling if nv else None),
        )
        lp = req.logprobs
        oo = OutputOptions(logprobs=(1 if lp is True else (lp or None)))
        return PreprocessedRequest(token_ids=token_ids, stop_conditions=sc, sampling_options=so, output_options=oo,
                                   eos_token_ids=self.eos, mdc_sum=self.mdc_sum,
                                   annotations=list(nv.annotations or []) if nv else [])

    def preprocess_chat(self, req: ChatCompletionRequest) -> tuple[PreprocessedRequest, dict]:
        nv = req.nvext
        msgs = [m.model_dump(exclude_none=True) for m in req.messages]
        images: list[str] = []
        for m in msgs:
            if isinstance(m.get("content"), list):
                parts = []
                for p in m["content"]:
                    if not isinstance(p, dict):
                        continue
                    if p.get("type") == "image_url" and self.image_token_id is not None:
                        url = p.get("image_url")
                        images.append(url.get("url") if isinstance(url, dict) else url)
                        parts.append(IMAGE_MARKER)
                    else:
                        parts.append(p.get("text", ""))
                m["content"] = "".join(parts)
        if nv and nv.use_raw_prompt:
            prompt = "".join(m.get("content") or "" for m in msgs)
        else:
            # reference oai.rs should_add_generation_prompt: only after a user turn
            # (a trailing assistant message is continued, not answered)
            gen = msgs[-1].get("role") == "user" if msgs else True
            prompt = self.formatter.render(msgs, tools=req.tools, add_generation_prompt=gen,
                                           **(req.chat_template_kwargs or {}))
        if images:
            # tokenize around the markers, splice image placeholder runs in
            ids = []
            for i, piece in enumerate(prompt.split(IMAGE_MARKER)):
                if i:
                    ids.extend([self.image_token_id] * self.image_tokens)
                if piece:
                    ids.extend(self.tok.encode(piece, add_special_tokens=False))
        else:
            ids = self.tok.encode(prompt, add_special_tokens=False)
        pre = self._common(req, ids)
        if images:
            pre.multi_modal = {"image_urls": images}
        return pre, {ANNOTATION_FORMATTED_PROMPT: prompt, ANNOTATION_TOKEN_IDS: ids}

    def preprocess_completion(self, req: CompletionRequest) -> tuple[PreprocessedRequest, dict]:
        p = req.prompt
        if isinstance(p, list) and p and isinstance(p[0], int):
            ids, text = list(p), None
        elif isinstance(p, list) and p and isinstance(p[0], list):
            ids, text = list(p[0]), None
        else:
            text = p if isinstance(p, str) else (p[0] if p else "")
            ids = self.tok.encode(text, add_special_tokens=True)
        pre = self._common(req, ids)
        return pre, {ANNOTATION_FORMATTED_PROMPT: text, ANNOTATION_TOKEN_IDS: ids}

    # ------------------------------------------------------------------ out
    async def chat_stream(self, req: ChatCompletionRequest, backend_stream: AsyncIterator[dict], ann: dict,
                          request_id: str | None = None) -> AsyncIterator[dict]:
        """Backend outputs -> chat.completion.chunk dicts (DeltaGenerator)."""
        rid = request_id or new_request_id()
        created = int(time.time())
        wanted = set(req.nvext.annotations or []) if req.nvext else set()
        for a in wanted:
            if a in ann:
                yield {"event": a, "comment": [str(ann[a])]}
        first = True
        n_out = 0
        prompt_tokens = len(ann.get(ANNOTATION_TOKEN_IDS) or [])
        model = req.model
        want_lp = bool(req.logprobs)
        # chunks are built as plain dicts, field for field what
        # ChatCompletionChunk(...).model_dump(exclude_none=True) gives: three
        # pydantic models per streamed token were the processor's top cost
        async for out in backend_stream:
            text = out.get("text") or ""
            n_out += len(out.get("token_ids") or [])
            fr = out.get("finish_reason")
            delta = {}
            if first:
                delta["role"] = "assistant"
            if text or first:
                delta["content"] = text
            choice = {"index": 0, "delta": delta}
            if fr:
                choice["finish_reason"] = FINISH_MAP.get(fr, fr)
            if want_lp and out.get("log_probs"):
                choice["logprobs"] = {"content": [{"token": t, "logprob": l} for t, l in
                                                  zip(out.get("tokens") or [""] * len(out["log_probs"]),
                                                      out["log_probs"])]}
            first = False
            yield {"id": rid, "object": "chat.completion.chunk", "created": created, "model": model,
                   "choices": [choice]}
        if req.stream_options and req.stream_options.include_usage:
            yield ChatCompletionChunk(id=rid, created=created, model=req.model, choices=[],
                                      usage=Usage(prompt_tokens=prompt_tokens, completion_tokens=n_out,
                                                  total_tokens=prompt_tokens + n_out)).model_dump(exclude_none=True)

    async def completion_stream(self, req: CompletionRequest, backend_stream: AsyncIterator[dict], ann: dict,
                                request_id: str | None = None) -> AsyncIterator[dict]:
        rid = request_id or new_request_id("cmpl")
        created = int(time.time())
        n_out = 0
        prompt_tokens = len(ann.get(ANNOTATION_TOKEN_IDS) or [])
        if req.echo and ann.get(ANNOTATION_FORMATTED_PROMPT):
            yield CompletionResponse(id=rid, created=created, model=req.model,
                                     choices=[CompletionChoice(text=ann[ANNOTATION_FORMATTED_PROMPT])]).model_dump()
        model = req.model
        async for out in backend_stream:
            n_out += len(out.get("token_ids") or [])
            fr = out.get("finish_reason")
            choice = {"index": 0, "text": out.get("text") or ""}
            if fr:
                choice["finish_reason"] = FINISH_MAP.get(fr, fr)
            yield {"id": rid, "object": "text_completion", "created": created, "model": model, "choices": [choice]}
        if req.stream_options and req.stream_options.include_usage:
            yield CompletionResponse(id=rid, created=created, model=req.model, choices=[],
                                     usage=Usage(prompt_tokens=prompt_tokens, completion_tokens=n_out,
                                                 total_tokens=prompt_tokens + n_out)).model_dump(exclude_none=True)


# --------------------------------------------------------------------- aggregators
async def aggregate_chat(stream: AsyncIterator[dict]) -> dict:
    """Fold chat chunks into a unary chat.completion (DeltaAggregator)."""
    rid, model, created = None, None, None
    text, finish, usage = [], None, None
    async for ch in stream:
        if "event" in ch and "choices" not in ch:
            continue
        rid, model, created = ch.get("id", rid), ch.get("model", model), ch.get("created", created)
        if ch.get("usage"):
            usage = ch["usage"]
        for c in ch.get("choices", []):
            d = c.get("delta", {})
            if d.get("content"):
                text.append(d["content"])
            if c.get("finish_reason"):
                finish = c["finish_reason"]
    return ChatCompletionResponse(id=rid or new_request_id(), created=created or int(time.time()), model=model or "",
                                  choices=[ChatChoice(message=ChatMessage(role="assistant", content="".join(text)),
                                                      finish_reason=finish)],
                                  usage=Usage(**usage) if usage else None).model_dump(exclude_none=True)


async def aggregate_completion(stream: AsyncIterator[dict]) -> dict:
    rid, model, created = None, None, None
    text, finish, usage = [], None, None
    async for ch in stream:
        rid, model, created = ch.get("id", rid), ch.get("model", model), ch.get("created", created)
        if ch.get("usage"):
            usage = ch["usage"]
        for c in ch.get("choices", []):
            text.append(c.get("text") or "")
            if c.get("finish_reason"):
                finish = c["finish_reason"]
    return CompletionResponse(id=rid or new_request_id("cmpl"), created=created or int(time.time()), model=model or "",
                              choices=[CompletionChoice(text="".join(text), finish_reason=finish)],
                              usage=Usage(**usage) if usage else None).model_dump(exclude_none=True)
