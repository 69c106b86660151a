"""HTTP routes around the serving path: the reference's FastAPI app
(app/main.py:30-196) — `/health`, `/`, `/recommend`, `/score`, `/model/info` with the same request /
response schemas, status codes (503 model not loaded, 404 unknown user on /score, 500 otherwise) and
startup loading — over `serving.RecommendationService` (the GPU index: user tower on the GEMM
kernels, L2 normalisation and exact top-k on the HIP kernels).

    uvicorn "recommendation-system-maang-nvidia-_amd.api:app"   (RS_MODEL_DIR, default
    outputs/models/experiment_001 as app/main.py:113)

`create_app(model_dir=None, service=None)` builds an app around a given directory or an already
loaded service (tests, embedding in another server)."""
from __future__ import annotations

import logging
import os
from contextlib import asynccontextmanager
from typing import Callable, Dict, List, Optional

from fastapi import FastAPI, HTTPException
from fastapi.middleware.cors import CORSMiddleware
from pydantic import BaseModel, Field

logger = logging.getLogger(__name__)


class RecommendationRequest(BaseModel):
    user_id: str = Field(..., description="User ID to get recommendations for")
    k: int = Field(10, ge=1, le=100, description="Number of recommendations to return")


class RecommendationItem(BaseModel):
    item_id: str
    score: float
    rank: int


class RecommendationResponse(BaseModel):
    user_id: str
    recommendations: List[RecommendationItem]
    count: int
    model_version: str


class ScoreRequest(BaseModel):
    user_id: str
    item_ids: List[str] = Field(..., min_length=1, max_length=100)


class ScoreResponse(BaseModel):
    user_id: str
    scores: Dict[str, float]


class HealthResponse(BaseModel):
    status: str
    model_loaded: bool
    model_version: Optional[str] = None


def _load_service(model_dir: str):
    from .serving import RecommendationService
    svc = RecommendationService(model_dir=model_dir)
    svc.load()
    return svc


def create_app(model_dir: Optional[str] = None, service=None,
               loader: Callable[[str], object] = _load_service) -> FastAPI:
    """The reference's routes over `service` (an object with is_ready / recommend / score /
    get_model_info), or over one `loader(model_dir)` builds at startup (a failed load leaves the
    routes answering 503, app/main.py:106-117)."""
    state = {"service": service}

    @asynccontextmanager
    async def lifespan(_app):
        # startup (app/main.py:106-117): load unless a service was given
        if state["service"] is None:
            path = model_dir or os.environ.get("RS_MODEL_DIR", "outputs/models/experiment_001")
            try:
                state["service"] = loader(path)
                logger.info("recommendation service loaded from %s", path)
            except Exception as e:  # the routes answer 503 (app/main.py:115-117)
                logger.error("failed to load the model at startup: %s", e)
        yield
        state["service"] = None  # shutdown

    app = FastAPI(title="Recommendation System API",
                  description="Two-Tower + DCN recommendations on the MI355X serving path.",
                  version="1.2.0", docs_url="/docs", redoc_url="/redoc", lifespan=lifespan)
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                       allow_headers=["*"])

    def ready():
        svc = state["service"]
        return svc if svc is not None and svc.is_ready() else None

    @app.get("/health", response_model=HealthResponse, tags=["Health"])
    async def health_check():
        svc = ready()
        return HealthResponse(status="healthy" if svc else "degraded", model_loaded=svc is not None,
                              model_version=svc.get_model_info()["version"] if svc else None)

    @app.get("/", tags=["Info"], include_in_schema=False)
    async def root():
        return {"message": "Welcome to the Recommendation System API", "status": "running",
                "documentation": "/docs"}

    @app.post("/recommend", response_model=RecommendationResponse, tags=["Recommendations"])
    async def get_recommendations(request: RecommendationRequest):
        svc = ready()
        if svc is None:
            raise HTTPException(status_code=503, detail="Model not loaded. Service is unavailable.")
        try:
            recs = svc.recommend(user_id=request.user_id, k=request.k)
            return RecommendationResponse(user_id=request.user_id, recommendations=recs, count=len(recs),
                                          model_version=svc.get_model_info()["version"])
        except ValueError as e:
            raise HTTPException(status_code=404, detail=str(e))
        except Exception as e:
            logger.error("recommendation for user %r failed: %s", request.user_id, e)
            raise HTTPException(status_code=500, detail="Internal server error")

    @app.post("/score", response_model=ScoreResponse, tags=["Scoring"])
    async def score_items(request: ScoreRequest):
        svc = ready()
        if svc is None:
            raise HTTPException(status_code=503, detail="Model not loaded. Service is unavailable.")
        try:
            return ScoreResponse(user_id=request.user_id, scores=svc.score(user_id=request.user_id,
                                                                           item_ids=request.item_ids))
        except ValueError as e:
            raise HTTPException(status_code=404, detail=str(e))
        except Exception as e:
            logger.error("scoring for user %r failed: %s", request.user_id, e)
            raise HTTPException(status_code=500, detail="Internal server error")

    @app.get("/model/info", tags=["Model"])
    async def get_model_info():
        svc = ready()
        if svc is None:
            raise HTTPException(status_code=503, detail="Model not loaded. Service is unavailable.")
        return svc.get_model_info()

    app.state.rs = state
    return app


app = create_app()
